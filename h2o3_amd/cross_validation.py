"""Client-side fold iterators (reference h2o-py h2o/cross_validation.py):
iterating yields (train mask, test mask) frames per fold."""
from __future__ import annotations


class H2OPartitionIterator:
    def __init__(self, n):
        if abs(n - int(n)) >= 1e-15:
            raise ValueError("n must be an integer")
        self.n, self.masks = int(n), None

    def __iter__(self):
        for test in self._test_masks():
            yield 1 - test, test

    def _test_masks(self):
        raise NotImplementedError


class H2OKFold(H2OPartitionIterator):
    def __init__(self, fr, n_folds=3, seed=-1):
        super().__init__(fr.nrows)
        self.n_folds, self.fr, self.seed, self.fold_assignments = n_folds, fr, seed, None

    def __len__(self):
        return self.n_folds

    def _assign(self):
        return self.fr.kfold_column(self.n_folds, self.seed)

    def _test_masks(self):
        if self.fold_assignments is None:
            self.fold_assignments = self._assign()
        if self.masks is None:
            self.masks = [self.fold_assignments == i for i in range(self.n_folds)]
        return self.masks


class H2OStratifiedKFold(H2OKFold):
    def __init__(self, y, n_folds=3, seed=-1):
        super().__init__(y, n_folds, seed)

    def _assign(self):
        return self.fr.stratified_kfold_column(self.n_folds, self.seed)

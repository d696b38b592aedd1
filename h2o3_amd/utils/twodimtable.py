"""H2OTwoDimTable / ConfusionMatrix value classes of the client API
(reference h2o-py h2o/two_dim_table.py, h2o/model/confusion_matrix.py)."""
from __future__ import annotations


class H2OTwoDimTable:
    def __init__(self, table_header=None, table_description=None, col_header=None, cell_values=None,
                 raw_cell_values=None, col_types=None, row_header=None, col_formats=None):
        self._table_header = table_header or ""
        self._table_description = table_description or ""
        self._col_header = list(col_header or [])
        self._cell_values = [list(r) for r in (cell_values if cell_values is not None else raw_cell_values or [])]
        self._col_types = list(col_types or [])

    @staticmethod
    def from_pandas(df, table_header=""):
        return H2OTwoDimTable(table_header, col_header=list(df.columns), cell_values=df.values.tolist())

    @property
    def cell_values(self):
        return self._cell_values

    @property
    def col_header(self):
        return self._col_header

    @property
    def col_types(self):
        return self._col_types

    @property
    def table_header(self):
        return self._table_header

    @property
    def table_description(self):
        return self._table_description

    def as_data_frame(self):
        import pandas as pd
        return pd.DataFrame(self._cell_values, columns=self._col_header)

    def __getitem__(self, item):
        j = self._col_header.index(item) if isinstance(item, str) else int(item)
        return [r[j] for r in self._cell_values]

    def show(self, header=True):
        if header:
            print(self._table_header)
        print(self.as_data_frame().to_string(index=False))

    def __repr__(self):
        return f"{self._table_header}\n{self.as_data_frame().to_string(index=False)}"


class ConfusionMatrix:
    """A confusion matrix as a two-dimensional table (rows actual, columns
    predicted, last column Error / Rate)."""

    ROUND = 4

    def __init__(self, cm, domains=None, table_header=None):
        if isinstance(cm, H2OTwoDimTable):
            self.table = cm
            return
        rows = [list(r) for r in cm]
        dom = list(domains) if domains is not None else [str(i) for i in range(len(rows))]
        cells = []
        for d, r in zip(dom, rows):
            tot = sum(r)
            err = (tot - r[dom.index(d)]) / tot if tot else 0.0
            cells.append([d] + r + [round(err, self.ROUND)])
        self.table = H2OTwoDimTable(table_header or "Confusion Matrix", col_header=[""] + dom + ["Error"],
                                    cell_values=cells)

    def to_list(self):
        return [[int(v) for v in r[1:-1]] for r in self.table.cell_values]

    def show(self):
        self.table.show()

    def __repr__(self):
        return repr(self.table)

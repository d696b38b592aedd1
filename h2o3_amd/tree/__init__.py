"""H2OTree: inspect one tree of a tree-based model.

Reference: h2o-py h2o/tree/tree.py (H2OTree / H2ONode / H2OSplitNode /
H2OLeafNode, fields left_children, right_children, node_ids, descriptions,
thresholds, features, levels, nas, predictions, root_node) backed by
hex/tree/TreeHandler.java.
"""
from __future__ import annotations

import math


class H2ONode:
    def __init__(self, node_id):
        self.id = node_id


class H2OLeafNode(H2ONode):
    def __init__(self, node_id, prediction):
        super().__init__(node_id)
        self.prediction = prediction

    def __repr__(self):
        return f"Leaf node ID {self.id}. Predicted value at leaf node is {self.prediction}"


class H2OSplitNode(H2ONode):
    def __init__(self, node_id, threshold, left, right, split_feature, na_direction, left_levels, right_levels):
        super().__init__(node_id)
        self.threshold, self.left_child, self.right_child = threshold, left, right
        self.split_feature, self.na_direction = split_feature, na_direction
        self.left_levels, self.right_levels = left_levels, right_levels

    def __repr__(self):
        return f"Node ID {self.id}: split on {self.split_feature} at {self.threshold}, NA -> {self.na_direction}"


class H2OTree:
    def __init__(self, model, tree_number, tree_class=None, plain_language_rules="AUTO"):
        K = model._n_tree_classes()
        dom = model._spec.response_domain
        if tree_class is not None and not isinstance(tree_class, int):
            tree_class = dom.index(tree_class)
        if K > 1 and tree_class is None:
            raise ValueError("tree_class must be specified for multinomial models")
        t = model.get_tree(tree_number, tree_class)
        names = list(model._spec.x)
        doms = getattr(model, "_x_domains", {})
        self.tree_number, self.tree_class = tree_number, tree_class
        self.model_id = model.model_id
        n = t.n_nodes
        self.node_ids = list(range(n))
        self.left_children = [t.left[i] for i in range(n)]
        self.right_children = [t.right[i] for i in range(n)]
        self.features, self.thresholds, self.nas, self.levels, self.predictions, self.descriptions = \
            [], [], [], [], [], []
        for i in range(n):
            leaf = t.left[i] < 0
            f = None if leaf else names[t.feat[i]]
            self.features.append(f)
            self.predictions.append(float(t.value[i]))
            if leaf:
                self.thresholds.append(float("nan"))
                self.nas.append(None)
                self.levels.append(None)
                self.descriptions.append(f"Leaf node, prediction {t.value[i]}")
                continue
            self.nas.append("LEFT" if t.na_left[i] else "RIGHT")
            if t.is_cat[i] and t.cat_left[i] is not None:
                dm = doms.get(f, [])
                self.thresholds.append(float("nan"))
                self.levels.append([dm[k] for k in range(min(len(dm), len(t.cat_left[i]))) if t.cat_left[i][k]])
                self.descriptions.append(f"Categorical split on {f}; left levels {self.levels[-1]}")
            else:
                self.thresholds.append(float(t.thr[i]))
                self.levels.append(None)
                self.descriptions.append(f"Numerical split on {f} < {t.thr[i]}; NA goes {self.nas[-1]}")
        self._t = t
        self.root_node = self._build(0)

    def _build(self, i):
        if self.left_children[i] < 0:
            return H2OLeafNode(i, self.predictions[i])
        l, r = self._build(self.left_children[i]), self._build(self.right_children[i])
        rl = None
        if self.levels[i] is not None:
            rl = None
        return H2OSplitNode(i, self.thresholds[i], l, r, self.features[i], self.nas[i], self.levels[i], rl)

    def __len__(self):
        return len(self.node_ids)

    def __repr__(self):
        return f"Tree related to model {self.model_id}. Tree number is {self.tree_number}, tree class is " \
               f"{self.tree_class}\n\nThe tree has {len(self)} nodes"

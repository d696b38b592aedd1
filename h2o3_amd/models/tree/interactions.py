"""Tree-ensemble introspection: feature interactions (XGBFI-style tables),
per-row feature frequencies and node re-weighting.

Reference:
  * hex/FeatureInteractions.java:225 collectFeatureInteractions — every
    split node opens an interaction path; paths are extended down both
    children up to max_interaction_depth, new paths may start below the
    root up to max_deepening; per interaction (features sorted by name,
    joined by "|"): Gain, FScore, wFScore (path probability), averages,
    Expected Gain, tree index / depth, leaf statistics of depth-0
    deepening, split value histograms of single features; tables ranked
    per metric (FeatureInteractions.constructFeatureInteractionsTable);
    hex/tree/gbm/GBMModel.java:283 (one collection per tree, merged);
  * feature_frequencies: number of times each feature is used on a row's
    decision path, summed over trees (Predictions ... feature_frequencies);
  * update_tree_weights: node covers recomputed from a frame with a weight
    column (SharedTreeModel.updateTreeWeights), which re-bases TreeSHAP.

The trees are small host-side structures, so the interaction collection is
host code; the per-row parts (leaf assignment, frequencies, weights) run on
the device through the forest scoring kernel's leaf ids.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch
from ...core.groupsum import index_add as _ia


class _FI:
    __slots__ = ("name", "depth", "gain", "cover", "fscore", "wfscore", "expected_gain", "tree_index",
                 "tree_depth", "has_leaf", "lv_left", "lc_left", "lv_right", "lc_right", "split_hist")

    def __init__(self, path_names, gain, cover, proba, depth, tree_index, split_value):
        self.name = "|".join(path_names)
        self.depth = len(path_names) - 1
        self.gain, self.cover, self.fscore, self.wfscore = gain, cover, 1.0, proba
        self.expected_gain = gain * proba
        self.tree_index, self.tree_depth = float(tree_index), float(depth)
        self.has_leaf = False
        self.lv_left = self.lc_left = self.lv_right = self.lc_right = 0.0
        self.split_hist = {}
        if self.depth == 0:
            self.split_hist[split_value] = 1

    def merge(self, o):
        self.gain += o.gain
        self.cover += o.cover
        self.fscore += o.fscore
        self.wfscore += o.wfscore
        self.expected_gain += o.expected_gain
        self.tree_index += o.tree_index
        self.tree_depth += o.tree_depth
        self.lv_left += o.lv_left
        self.lc_left += o.lc_left
        self.lv_right += o.lv_right
        self.lc_right += o.lc_right
        self.has_leaf = self.has_leaf or o.has_leaf
        for k, v in o.split_hist.items():
            self.split_hist[k] = self.split_hist.get(k, 0) + v


def _collect(tree, names, node, path, cur_gain, cur_cover, proba, depth, deepening, acc, memo, max_id, max_td,
             max_deep, tree_index):
    if tree.left[node] < 0 or depth == max_td:
        return
    path = path + [node]
    cur_gain += float(tree.gain[node])
    cur_cover += float(tree.weight[node])
    L, R = tree.left[node], tree.right[node]
    w = float(tree.weight[node]) or 1e-300
    ppl = proba * (float(tree.weight[L]) / w)
    ppr = proba * (float(tree.weight[R]) / w)
    # features sorted by name (stable), like interactionPathToStr(.., sortByFeature)
    path.sort(key=lambda n: names[tree.feat[n]])
    fi = _FI([names[tree.feat[n]] for n in path], cur_gain, cur_cover, proba, depth, tree_index,
             float(tree.thr[path[0]]))
    if depth < max_deep or max_deep < 0:
        _collect(tree, names, L, [], 0.0, 0.0, ppl, depth + 1, deepening + 1, acc, memo, max_id, max_td, max_deep,
                 tree_index)
        _collect(tree, names, R, [], 0.0, 0.0, ppr, depth + 1, deepening + 1, acc, memo, max_id, max_td, max_deep,
                 tree_index)
    key = "-".join(str(n) for n in path)
    found = acc.get(fi.name)
    if found is None:
        acc[fi.name] = fi
        memo.add(key)
    else:
        if key in memo:
            return
        memo.add(key)
        found.merge(fi)
    if len(path) - 1 == max_id:
        return
    found = acc[fi.name]
    if tree.left[L] < 0 and deepening == 0:
        found.lv_left += float(tree.value[L])
        found.lc_left += float(tree.weight[L])
        found.has_leaf = True
    if tree.left[R] < 0 and deepening == 0:
        found.lv_right += float(tree.value[R])
        found.lc_right += float(tree.weight[R])
        found.has_leaf = True
    # the reference passes the accumulated gain as the cover of the extended path
    _collect(tree, names, L, list(path), cur_gain, cur_gain, ppl, depth + 1, deepening, acc, memo, max_id, max_td,
             max_deep, tree_index)
    _collect(tree, names, R, list(path), cur_gain, cur_gain, ppr, depth + 1, deepening, acc, memo, max_id, max_td,
             max_deep, tree_index)


def feature_interactions(forest, names, ntrees_per_class, K, max_interaction_depth=100, max_tree_depth=100,
                         max_deepening=-1):
    """Merged FeatureInteractions of every tree -> dict name -> _FI."""
    total = {}
    for t, tree in enumerate(forest.trees):
        acc, memo = {}, set()
        _collect(tree, names, 0, [], 0.0, 0.0, 1.0, 0, 0, acc, memo, int(max_interaction_depth),
                 int(max_tree_depth), int(max_deepening), t // max(K, 1))
        for k, v in acc.items():
            if k in total:
                total[k].merge(v)
            else:
                total[k] = v
    return total


def interaction_tables(fis):
    """[one table per interaction depth] + [leaf statistics] + [split value
    histograms of single features], as pandas DataFrames."""
    if not fis:
        return []
    out = []
    max_depth = max(f.depth for f in fis.values())
    for d in range(max_depth + 1):
        rows = [f for f in fis.values() if f.depth == d]
        df = pd.DataFrame({"Interaction": [f.name for f in rows], "Gain": [f.gain for f in rows],
                           "FScore": [f.fscore for f in rows], "wFScore": [f.wfscore for f in rows],
                           "Average wFScore": [f.wfscore / f.fscore for f in rows],
                           "Average Gain": [f.gain / f.fscore for f in rows],
                           "Expected Gain": [f.expected_gain for f in rows]})
        for col, rank in (("Gain", "Gain Rank"), ("FScore", "FScore Rank"), ("wFScore", "wFScore Rank"),
                          ("Average wFScore", "Avg wFScore Rank"), ("Average Gain", "Avg Gain Rank"),
                          ("Expected Gain", "Expected Gain Rank")):
            order = sorted(range(len(rows)), key=lambda i: -df[col].iloc[i])
            r = np.empty(len(rows), dtype=np.int64)
            r[order] = np.arange(1, len(rows) + 1)
            df[rank] = r
        df["Average Rank"] = df[[c for c in df.columns if c.endswith("Rank")]].mean(1)
        df["Average Tree Index"] = [f.tree_index / f.fscore for f in rows]
        df["Average Tree Depth"] = [f.tree_depth / f.fscore for f in rows]
        df.attrs["table_header"] = f"Interaction Depth {d}"
        out.append(df)
    leaf = [f for f in fis.values() if f.has_leaf]
    ls = pd.DataFrame({"Interaction": [f.name for f in leaf], "Sum Leaf Values Left": [f.lv_left for f in leaf],
                       "Sum Leaf Values Right": [f.lv_right for f in leaf],
                       "Sum Leaf Covers Left": [f.lc_left for f in leaf],
                       "Sum Leaf Covers Right": [f.lc_right for f in leaf]})
    ls.attrs["table_header"] = "Leaf Statistics"
    out.append(ls)
    for f in fis.values():
        if f.depth == 0:
            h = pd.DataFrame({"Split Value": list(f.split_hist.keys()), "Count": list(f.split_hist.values())})
            h.attrs["table_header"] = f"{f.name} Split Value Histogram"
            out.append(h)
    return out


def _path_feature_counts(tree, F):
    """[n_nodes, F] number of times each feature splits on the path root -> node."""
    cnt = np.zeros((tree.n_nodes, F), dtype=np.float32)
    stack = [0]
    while stack:
        n = stack.pop()
        if tree.left[n] >= 0:
            for c in (tree.left[n], tree.right[n]):
                cnt[c] = cnt[n]
                cnt[c, tree.feat[n]] += 1
                stack.append(c)
    return cnt


def feature_frequencies(forest, leaf_ids: torch.Tensor, F: int) -> torch.Tensor:
    """leaf_ids [n, T] (tree-local node ids) -> [n, F] feature use counts."""
    out = torch.zeros((leaf_ids.shape[0], F), dtype=torch.float32, device=leaf_ids.device)
    for t, tree in enumerate(forest.trees):
        cnt = torch.as_tensor(_path_feature_counts(tree, F), device=leaf_ids.device)
        out += cnt.index_select(0, leaf_ids[:, t].long())
    return out


def update_tree_weights(forest, leaf_ids: torch.Tensor, w: torch.Tensor):
    """Node covers = sum of the row weights reaching each node."""
    for t, tree in enumerate(forest.trees):
        leaf_w = torch.zeros(tree.n_nodes, dtype=torch.float64, device=leaf_ids.device)
        _ia(leaf_w, leaf_ids[:, t].long(), w.to(torch.float64))
        from ...parallel import collectives as coll
        coll.allreduce_(leaf_w)
        wt = leaf_w.cpu().numpy()
        # internal nodes: children come after their parent in BFS order
        for n in range(tree.n_nodes - 1, -1, -1):
            if tree.left[n] >= 0:
                wt[n] = wt[tree.left[n]] + wt[tree.right[n]]
        tree.weight = [float(x) for x in wt]
    forest._packed = None

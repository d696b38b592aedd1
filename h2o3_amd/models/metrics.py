"""Model metrics computed on device.

Reference: hex/ModelMetrics*.java, hex/AUC2.java (threshold table with up
to 400 bins; AUC via trapezoids), hex/ConfusionMatrix.java,
hex/GainsLift.java, hex/MultinomialAUC.java, hex/ModelMetricsClustering.java.

The reference builds metrics with an MRTask of per-row updates into
AUC2 histograms; here the scores and labels live in HBM, so the binomial
metrics come from one GPU sort (exact AUC) plus a 400-point threshold table
for the confusion-matrix family, all-gathered when sharded.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from ..core.groupsum import index_add as _ia

_MAX_THRESHOLDS = 400


def _gather(t):
    return coll.all_gather_var(t) if cloud.is_distributed() else t


class ModelMetrics:
    kind = "base"

    def __init__(self, **kw):
        self._m = dict(kw)

    def __getitem__(self, k):
        return self._m[k]

    def get(self, k, d=None):
        return self._m.get(k, d)

    def _metric(self, k):
        return self._m.get(k)

    # common accessors (h2o-py ModelMetricsBase)
    def mse(self): return self._m.get("MSE")
    def rmse(self): return self._m.get("RMSE")
    def mae(self): return self._m.get("mae")
    def rmsle(self): return self._m.get("rmsle")
    def r2(self): return self._m.get("r2")
    def logloss(self): return self._m.get("logloss")
    def auc(self): return self._m.get("AUC")
    def aucpr(self): return self._m.get("pr_auc")
    pr_auc = aucpr
    def gini(self): return self._m.get("Gini")
    def mean_per_class_error(self): return self._m.get("mean_per_class_error")
    def mean_residual_deviance(self): return self._m.get("mean_residual_deviance")
    def nobs(self): return self._m.get("nobs")
    def null_deviance(self): return self._m.get("null_deviance")
    def residual_deviance(self): return self._m.get("residual_deviance")
    def aic(self): return self._m.get("AIC")
    def custom_metric_value(self): return self._m.get("custom_metric_value")

    def confusion_matrix(self, metrics=None, thresholds=None):
        return self._m.get("cm")

    def metric(self, name, thresholds=None):
        tt = self._m.get("thresholds_and_metric_scores")
        if tt is None:
            return None
        if thresholds is None:
            i = int(np.argmax(tt[name]))
            return [[tt["threshold"][i], tt[name][i]]]
        out = []
        for t in thresholds:
            i = int(np.argmin(np.abs(np.asarray(tt["threshold"]) - t)))
            out.append([t, tt[name][i]])
        return out

    def find_threshold_by_max_metric(self, metric):
        tt = self._m["thresholds_and_metric_scores"]
        return float(tt["threshold"][int(np.argmax(tt[metric]))])

    def F1(self, thresholds=None): return self.metric("f1", thresholds)
    def F2(self, thresholds=None): return self.metric("f2", thresholds)
    def F0point5(self, thresholds=None): return self.metric("f0point5", thresholds)
    def accuracy(self, thresholds=None): return self.metric("accuracy", thresholds)
    def precision(self, thresholds=None): return self.metric("precision", thresholds)
    def recall(self, thresholds=None): return self.metric("recall", thresholds)
    sensitivity = recall
    def tpr(self, thresholds=None): return self.metric("tpr", thresholds)
    def tnr(self, thresholds=None): return self.metric("tnr", thresholds)
    def fnr(self, thresholds=None): return self.metric("fnr", thresholds)
    def fpr(self, thresholds=None): return self.metric("fpr", thresholds)
    fallout = fpr
    missrate = fnr
    def specificity(self, thresholds=None): return self.metric("specificity", thresholds)
    def mcc(self, thresholds=None): return self.metric("absolute_mcc", thresholds)

    def error(self, thresholds=None):
        acc = self.metric("accuracy", thresholds)
        return None if acc is None else [[t, 1 - a] for t, a in acc]

    def max_per_class_error(self, thresholds=None):
        m = self.metric("min_per_class_accuracy", thresholds)
        return None if m is None else [[t, 1 - a] for t, a in m]

    def thresholds_and_metric_scores(self):
        import pandas as pd
        tt = self._m.get("thresholds_and_metric_scores")
        return None if tt is None else pd.DataFrame(tt)

    def thresholds(self):
        tt = self._m.get("thresholds_and_metric_scores")
        return None if tt is None else list(tt["threshold"])

    def find_idx_by_threshold(self, threshold):
        tt = self._m["thresholds_and_metric_scores"]
        return int(np.argmin(np.abs(np.asarray(tt["threshold"]) - threshold)))

    def roc(self):
        """(fpr list, tpr list) over the threshold table."""
        tt = self._m.get("thresholds_and_metric_scores")
        return None if tt is None else (list(tt["fpr"]), list(tt["tpr"]))

    def kolmogorov_smirnov(self):
        """max(tpr - fpr) over thresholds (GainsLift KS of the reference)."""
        tt = self._m.get("thresholds_and_metric_scores")
        return None if tt is None else float(np.max(np.asarray(tt["tpr"]) - np.asarray(tt["fpr"])))

    def gains_lift(self):
        return self._m.get("gains_lift_table")

    def hit_ratio_table(self):
        return self._m.get("hit_ratio_table")

    def tot_withinss(self): return self._m.get("tot_withinss")
    def betweenss(self): return self._m.get("betweenss")
    def totss(self): return self._m.get("totss")
    def withinss(self): return self._m.get("withinss")

    def as_dict(self):
        return {k: v for k, v in self._m.items() if not isinstance(v, (dict, list, np.ndarray)) or k == "cm"}

    def __repr__(self):
        keys = [k for k, v in self._m.items() if isinstance(v, (int, float)) and v is not None]
        body = ", ".join(f"{k}={self._m[k]:.6g}" for k in keys)
        return f"ModelMetrics{self.kind.capitalize()}({body})"

    def show(self):
        print(repr(self))


class ModelMetricsRegression(ModelMetrics):
    kind = "regression"


class ModelMetricsBinomial(ModelMetrics):
    kind = "binomial"


class ModelMetricsMultinomial(ModelMetrics):
    kind = "multinomial"

    def multinomial_auc_table(self):
        return self._m.get("multinomial_auc_table")

    def multinomial_aucpr_table(self):
        return self._m.get("multinomial_aucpr_table")


class ModelMetricsOrdinal(ModelMetricsMultinomial):
    kind = "ordinal"


class ModelMetricsClustering(ModelMetrics):
    kind = "clustering"


class ModelMetricsAnomaly(ModelMetrics):
    kind = "anomaly"


class ModelMetricsAutoEncoder(ModelMetrics):
    kind = "autoencoder"


class ModelMetricsDimReduction(ModelMetrics):
    kind = "dimreduction"


class ModelMetricsCoxPH(ModelMetrics):
    kind = "coxph"

    def concordance(self):
        return self._m.get("concordance")


class ModelMetricsUplift(ModelMetrics):
    kind = "binomial_uplift"

    def auuc(self, metric=None):
        return self._m.get("AUUC")

    def qini(self):
        return self._m.get("qini")


def _wsum(x):
    return coll.allreduce_scalar(float(x.sum()))


def regression_metrics(y, pred, w=None, distribution=None):
    ok = ~torch.isnan(y) & ~torch.isnan(pred)
    y, pred = y[ok].to(torch.float64), pred[ok].to(torch.float64)
    w = torch.ones_like(y) if w is None else w[ok].to(torch.float64)
    sw = _wsum(w)
    err = pred - y
    mse = _wsum(w * err * err) / sw if sw > 0 else float("nan")
    mae = _wsum(w * err.abs()) / sw if sw > 0 else float("nan")
    ymean = _wsum(w * y) / sw if sw > 0 else float("nan")
    var = _wsum(w * (y - ymean) ** 2) / sw if sw > 0 else float("nan")
    r2 = 1 - mse / var if var and var > 0 else float("nan")
    # the rmsle domain check is agreed over ranks (a rank-local test would
    # leave the ranks issuing different collectives)
    bad = _wsum(((y <= -1) | (pred <= -1)).to(torch.float64))
    if bad == 0 and sw > 0:
        rmsle = math.sqrt(_wsum(w * (torch.log1p(pred) - torch.log1p(y)) ** 2) / sw)
    else:
        rmsle = float("nan")
    if sw <= 0:
        dev = float("nan")
    elif distribution is not None and distribution.family not in ("gaussian",):
        dev = _wsum(distribution.deviance(w, y, pred)) / sw
    else:
        dev = mse
    n = int(coll.allreduce_scalar(float(y.numel())))
    return ModelMetricsRegression(MSE=mse, RMSE=math.sqrt(mse) if mse == mse else float("nan"), mae=mae,
                                  rmsle=rmsle, r2=r2, mean_residual_deviance=dev, nobs=n)


def _auc_exact(p, y, w):
    """Weighted ROC AUC via a single sort (ties averaged)."""
    order = torch.argsort(p, descending=True)
    ps, ys, ws = p[order], y[order], w[order]
    tp = torch.cumsum(ws * ys, 0)
    fp = torch.cumsum(ws * (1 - ys), 0)
    # keep last index of each tie group
    last = torch.ones_like(ps, dtype=torch.bool)
    if ps.numel() > 1:
        last[:-1] = ps[1:] != ps[:-1]
    tp, fp = tp[last], fp[last]
    P, N = tp[-1], fp[-1]
    if P <= 0 or N <= 0:
        return float("nan"), float("nan")
    tpr = torch.cat([torch.zeros(1, dtype=tp.dtype, device=tp.device), tp / P])
    fpr = torch.cat([torch.zeros(1, dtype=fp.dtype, device=fp.device), fp / N])
    auc = float(torch.trapz(tpr, fpr))
    # PR AUC (average precision style trapezoid over recall)
    prec = tp / (tp + fp).clamp_min(1e-300)
    rec = tp / P
    rec0 = torch.cat([torch.zeros(1, dtype=rec.dtype, device=rec.device), rec])
    prec0 = torch.cat([prec[:1], prec])
    prauc = float(torch.trapz(prec0, rec0))
    return auc, prauc


def _threshold_table(p, y, w):
    """Confusion-matrix family over <=400 thresholds (AUC2-style)."""
    P = float((w * y).sum())
    N = float((w * (1 - y)).sum())
    u = torch.unique(p)
    if u.numel() > _MAX_THRESHOLDS:
        q = torch.linspace(0, 1, _MAX_THRESHOLDS, dtype=torch.float64, device=p.device)
        srt = torch.sort(p).values
        u = torch.unique(srt[(q * (srt.numel() - 1)).long()])
    thr = torch.sort(u, descending=True).values
    # counts of predictions >= thr
    srt_idx = torch.argsort(p)
    ps = p[srt_idx]
    cw_pos = torch.cumsum((w * y)[srt_idx].flip(0), 0).flip(0)
    cw_neg = torch.cumsum((w * (1 - y))[srt_idx].flip(0), 0).flip(0)
    pos_idx = torch.searchsorted(ps, thr, right=False)
    n = ps.numel()
    valid = pos_idx < n
    tp = torch.where(valid, cw_pos[pos_idx.clamp(max=n - 1)], torch.zeros_like(thr))
    fp = torch.where(valid, cw_neg[pos_idx.clamp(max=n - 1)], torch.zeros_like(thr))
    fn = P - tp
    tn = N - fp
    eps = 1e-300
    prec = tp / (tp + fp).clamp_min(eps)
    rec = tp / max(P, eps)
    spec = tn / max(N, eps)
    acc = (tp + tn) / max(P + N, eps)

    def fb(b):
        return (1 + b * b) * prec * rec / (b * b * prec + rec).clamp_min(eps)
    mcc_den = torch.sqrt(((tp + fp) * (tp + fn) * (tn + fp) * (tn + fn)).clamp_min(eps))
    mcc = ((tp * tn - fp * fn) / mcc_den).abs()
    tpr, fpr = rec, fp / max(N, eps)
    tnr, fnr = spec, fn / max(P, eps)
    mpca = (tpr + tnr) / 2
    mina = torch.minimum(tpr, tnr)
    tab = {"threshold": thr, "f1": fb(1.0), "f2": fb(2.0), "f0point5": fb(0.5), "accuracy": acc,
           "precision": prec, "recall": rec, "specificity": spec, "absolute_mcc": mcc,
           "min_per_class_accuracy": mina, "mean_per_class_accuracy": mpca, "tns": tn, "fns": fn, "fps": fp,
           "tps": tp, "tnr": tnr, "fnr": fnr, "fpr": fpr, "tpr": tpr}
    return {k: v.cpu().numpy() for k, v in tab.items()}


def _gains_lift(p, y, w, groups=16):
    order = torch.argsort(p, descending=True)
    ys, ws = (y * w)[order], w[order]
    cw = torch.cumsum(ws, 0)
    tot = float(cw[-1])
    P = float(ys.sum())
    rows = []
    prev = 0
    cum_resp = 0.0
    for g in range(1, groups + 1):
        frac = g / groups
        idx = int(torch.searchsorted(cw, torch.tensor([frac * tot], dtype=cw.dtype, device=cw.device)).item())
        idx = min(max(idx, prev), ys.numel() - 1)
        grp_resp = float(ys[prev: idx + 1].sum())
        grp_w = float(ws[prev: idx + 1].sum())
        cum_resp += grp_resp
        resp_rate = grp_resp / grp_w if grp_w > 0 else 0
        avg = P / tot if tot > 0 else 0
        rows.append({"group": g, "cumulative_data_fraction": frac,
                     "lower_threshold": float(p[order][idx]), "lift": resp_rate / avg if avg > 0 else 0,
                     "cumulative_lift": (cum_resp / float(cw[idx])) / avg if avg > 0 else 0,
                     "response_rate": resp_rate, "cumulative_capture_rate": cum_resp / P if P > 0 else 0})
        prev = idx + 1
        if prev >= ys.numel():
            break
    return rows


# ---------------------------------------------------------------- sketches
# Mergeable score sketch (the role of hex/AUC2.java's 400-bin AUCBuilder,
# which is merged across nodes in MRTask.reduce): per-rank weighted
# histograms of positives / negatives over the score's logit, summed by one
# all-reduce.  Bins are uniform in logit space, so resolution holds at
# probabilities near 0 and 1; AUC, PR-AUC, the threshold table and the
# gains/lift groups are read off the merged histogram (ties within a bin
# are ties, as in AUC2's bins).  No row ever leaves its rank.
_NB_BIN = 1 << 18
_NB_MULTI = 2048
_LOGIT_LIM = 40.0


def _logit_bins(p, nb):
    p = p.to(torch.float64)
    x = (torch.log(p.clamp_min(1e-300)) - torch.log1p(-p.clamp_max(1.0 - 1e-16))).clamp(-_LOGIT_LIM, _LOGIT_LIM)
    return ((x + _LOGIT_LIM) * (nb / (2 * _LOGIT_LIM))).to(torch.int64).clamp(0, nb - 1)


def _bin_lower_prob(nb, device):
    x = -_LOGIT_LIM + torch.arange(nb, dtype=torch.float64, device=device) * (2 * _LOGIT_LIM / nb)
    return torch.sigmoid(x)


def _hist_auc(pos, neg):
    """(ROC AUC, PR AUC) from binned positives / negatives (ascending score)."""
    tp = torch.cumsum(pos.flip(0), 0)
    fp = torch.cumsum(neg.flip(0), 0)
    keep = (pos.flip(0) + neg.flip(0)) > 0
    tp, fp = tp[keep], fp[keep]
    if tp.numel() == 0:
        return float("nan"), float("nan")
    P, N = tp[-1], fp[-1]
    if P <= 0 or N <= 0:
        return float("nan"), float("nan")
    z = torch.zeros(1, dtype=tp.dtype, device=tp.device)
    auc = float(torch.trapz(torch.cat([z, tp / P]), torch.cat([z, fp / N])))
    prec = tp / (tp + fp).clamp_min(1e-300)
    rec = tp / P
    prauc = float(torch.trapz(torch.cat([prec[:1], prec]), torch.cat([z, rec])))
    return auc, prauc


def _threshold_table_hist(pos, neg, lower):
    """The confusion-matrix family at <= 400 thresholds (bin lower edges
    chosen by equal steps of cumulative weight, descending score)."""
    pd_, nd_ = pos.flip(0), neg.flip(0)
    thr_all = lower.flip(0)
    tp_all, fp_all = torch.cumsum(pd_, 0), torch.cumsum(nd_, 0)
    keep = torch.nonzero((pd_ + nd_) > 0).flatten()
    if keep.numel() > _MAX_THRESHOLDS:
        cw = (tp_all + fp_all)[keep]
        q = torch.linspace(0, float(cw[-1]), _MAX_THRESHOLDS, dtype=torch.float64, device=cw.device)
        sel = torch.unique(torch.searchsorted(cw, q).clamp(max=keep.numel() - 1))
        keep = keep[sel]
    thr, tp, fp = thr_all[keep], tp_all[keep], fp_all[keep]
    P, N = float(tp_all[-1]), float(fp_all[-1])
    return _cm_family(thr, tp, fp, P, N)


def _cm_family(thr, tp, fp, P, N):
    fn = P - tp
    tn = N - fp
    eps = 1e-300
    prec = tp / (tp + fp).clamp_min(eps)
    rec = tp / max(P, eps)
    spec = tn / max(N, eps)
    acc = (tp + tn) / max(P + N, eps)

    def fb(b):
        return (1 + b * b) * prec * rec / (b * b * prec + rec).clamp_min(eps)
    mcc_den = torch.sqrt(((tp + fp) * (tp + fn) * (tn + fp) * (tn + fn)).clamp_min(eps))
    mcc = ((tp * tn - fp * fn) / mcc_den).abs()
    tpr, fpr = rec, fp / max(N, eps)
    tnr, fnr = spec, fn / max(P, eps)
    tab = {"threshold": thr, "f1": fb(1.0), "f2": fb(2.0), "f0point5": fb(0.5), "accuracy": acc,
           "precision": prec, "recall": rec, "specificity": spec, "absolute_mcc": mcc,
           "min_per_class_accuracy": torch.minimum(tpr, tnr), "mean_per_class_accuracy": (tpr + tnr) / 2,
           "tns": tn, "fns": fn, "fps": fp, "tps": tp, "tnr": tnr, "fnr": fnr, "fpr": fpr, "tpr": tpr}
    return {k: v.cpu().numpy() for k, v in tab.items()}


def _gains_lift_hist(pos, neg, lower, groups=16):
    """hex/GainsLift.java groups off the merged histogram (descending score)."""
    pd_, nd_ = pos.flip(0).cpu().numpy(), neg.flip(0).cpu().numpy()
    thr = lower.flip(0).cpu().numpy()
    wd = pd_ + nd_
    cw = np.cumsum(wd)
    tot, P = float(cw[-1]) if cw.size else 0.0, float(pd_.sum())
    if tot <= 0:
        return []
    cresp = np.cumsum(pd_)
    avg = P / tot
    rows, prev, cum_prev = [], -1, 0.0
    for g in range(1, groups + 1):
        frac = g / groups
        idx = int(min(np.searchsorted(cw, frac * tot), cw.size - 1))
        if idx <= prev:
            continue
        grp_w = cw[idx] - (cw[prev] if prev >= 0 else 0.0)
        grp_r = cresp[idx] - (cresp[prev] if prev >= 0 else 0.0)
        rr = grp_r / grp_w if grp_w > 0 else 0.0
        rows.append({"group": g, "cumulative_data_fraction": float(cw[idx] / tot), "lower_threshold": float(thr[idx]),
                     "lift": rr / avg if avg > 0 else 0.0,
                     "cumulative_lift": (cresp[idx] / cw[idx]) / avg if avg > 0 and cw[idx] > 0 else 0.0,
                     "response_rate": rr, "cumulative_capture_rate": cresp[idx] / P if P > 0 else 0.0})
        prev = idx
    return rows


def _binomial_sketch(y, p1, w):
    """Merged [2, NB] positive / negative weight histograms over all ranks."""
    b = _logit_bins(p1, _NB_BIN)
    H = torch.zeros(2 * _NB_BIN, dtype=torch.float64, device=p1.device)
    H.index_add_(0, b + _NB_BIN * (1 - y).to(torch.int64), w)
    coll.allreduce_(H)
    return H[:_NB_BIN], H[_NB_BIN:]


def binomial_metrics(y, p1, w=None, domain=None, threshold=None, auc_type="AUTO", gainslift=True,
                     gainslift_bins=-1):
    """y in {0,1} (float), p1 = P(class 1).  AUC / PR-AUC / thresholds /
    gains-lift from the merged logit-histogram sketch (no gather of rows; a
    2^18-bin logit grid keeps the AUC within ~1e-5 of the exact sort)."""
    import os
    exact = os.environ.get("H2O3_EXACT_AUC") == "1" and not cloud.is_distributed()
    from ..ops import metrics_ops
    if not exact and metrics_ops.available(p1):
        # one HIP pass: NaN filter, logit sketch and the loss sums, one
        # all-reduce and one host read (ops/csrc/metrics.hip)
        buf = metrics_ops.logit_hist(y, p1, w, _NB_BIN)
        coll.allreduce_(buf)
        pos, neg = buf[:_NB_BIN], buf[_NB_BIN:2 * _NB_BIN]
        sw, ll_s, se_s, wy_s, nobs = (float(v) for v in buf[2 * _NB_BIN:].cpu().tolist())
    else:
        ok = ~torch.isnan(y) & ~torch.isnan(p1)
        y, p1 = y[ok].to(torch.float64), p1[ok].to(torch.float64)
        w = torch.ones_like(y) if w is None else w[ok].to(torch.float64)
        pc = torch.clamp(p1, 1e-15, 1 - 1e-15)
        sums = torch.stack([w.sum(), -(w * (y * torch.log(pc) + (1 - y) * torch.log(1 - pc))).sum(),
                            (w * (y - p1) ** 2).sum(), (w * y).sum(),
                            torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device)])
        coll.allreduce_(sums)
        sw, ll_s, se_s, wy_s, nobs = (float(v) for v in sums.cpu().tolist())
        pos = neg = None
    logloss = ll_s / sw if sw > 0 else float("nan")
    mse = se_s / sw if sw > 0 else float("nan")
    groups = 16 if gainslift_bins is None or int(gainslift_bins) < 0 else int(gainslift_bins)
    # the same merged sketch at every cloud size: metrics do not depend on
    # how many GPUs hold the rows (exact sort: H2O3_EXACT_AUC=1, one rank)
    if exact:
        auc, prauc = _auc_exact(p1, y, w)
        tab = _threshold_table(p1, y, w)
        gl = (lambda: _gains_lift(p1, y, w, groups)) if groups > 0 else None
    else:
        if pos is None:
            pos, neg = _binomial_sketch(y, p1, w)
        lower = _bin_lower_prob(_NB_BIN, pos.device)
        # only the occupied bins matter (cumulative sums, thresholds and
        # gains/lift groups are unchanged by empty bins): ONE device->host
        # copy of those, then the tables are built on the host
        nz = torch.nonzero((pos + neg) > 0).flatten()
        c = torch.stack([pos[nz], neg[nz], lower[nz]]).cpu()
        pos, neg, lower = c[0], c[1], c[2]
        auc, prauc = _hist_auc(pos, neg)
        tab = _threshold_table_hist(pos, neg, lower)
        gl = (lambda: _gains_lift_hist(pos, neg, lower, groups)) if groups > 0 else None
    i = int(np.argmax(tab["f1"])) if len(tab["f1"]) else 0
    thr = float(tab["threshold"][i]) if threshold is None and len(tab["threshold"]) else (threshold or 0.5)
    if threshold is not None:
        i = int(np.argmin(np.abs(tab["threshold"] - threshold)))
    tn, fp, fn, tp = (float(tab[k][i]) for k in ("tns", "fps", "fns", "tps"))
    P, N = tp + fn, tn + fp
    err0 = fp / N if N > 0 else 0
    err1 = fn / P if P > 0 else 0
    dom = domain or ["0", "1"]
    cm = {"domain": dom, "matrix": [[tn, fp], [fn, tp]], "threshold": thr,
          "errors": [err0, err1], "total_error": (fp + fn) / max(P + N, 1e-300)}
    ymean = wy_s / sw if sw > 0 else float("nan")
    var = ymean * (1 - ymean)
    m = ModelMetricsBinomial(MSE=mse, RMSE=math.sqrt(mse), logloss=logloss, AUC=auc, pr_auc=prauc,
                             Gini=2 * auc - 1 if auc == auc else float("nan"),
                             mean_per_class_error=(err0 + err1) / 2, max_f1_threshold=thr,
                             r2=1 - mse / var if var > 0 else float("nan"), nobs=int(nobs),
                             cm=cm, thresholds_and_metric_scores=tab, domain=dom)
    if gainslift and gl is not None:
        try:
            m._m["gains_lift_table"] = gl()
        except (RuntimeError, ValueError, IndexError):
            pass
    return m


_AUC_TYPES = ("AUTO", "NONE", "MACRO_OVR", "WEIGHTED_OVR", "MACRO_OVO", "WEIGHTED_OVO")
MAX_AUC_CLASSES = 50       # hex/MultinomialAUC.java MAX_AUC_CLASSES


def _auc_type(t):
    u = str(t or "AUTO").upper()
    if u not in _AUC_TYPES:
        raise ValueError(f"auc_type must be one of {list(_AUC_TYPES)}, got {t}")
    return u


def multinomial_auc(y, P, w, domain, auc_type):
    """hex/MultinomialAUC.java: one-vs-rest AUC per class, pairwise
    (one-vs-one) AUCs averaged over both directions (PairwiseAUC), and the
    macro / weighted aggregates, from one merged [K score classes, K true
    classes, bins] logit histogram (ModelMetricsMultinomial
    calculateAucsPerRow adds exactly these per-row terms to its AUC2
    builders).  Returns None when auc_type is AUTO / NONE or K > 50."""
    t = _auc_type(auc_type)
    K = P.shape[1]
    if t in ("AUTO", "NONE") or K > MAX_AUC_CLASSES:
        return None
    B = _NB_MULTI
    b = _logit_bins(P, B)                                     # [n, K] bin of p_s per row
    s_idx = torch.arange(K, device=P.device).view(1, K)
    idx = (s_idx * K + y.view(-1, 1)) * B + b
    H = torch.zeros(K * K * B, dtype=torch.float64, device=P.device)
    _ia(H, idx.reshape(-1), w.view(-1, 1).expand(-1, K).reshape(-1))
    coll.allreduce_(H)
    H = H.view(K, K, B)                                       # [score class, true class, bin]
    cls_w = H[0].sum(1).cpu().numpy()                         # weight of each true class
    n = float(cls_w.sum())
    ovr = []
    for i in range(K):
        pos = H[i, i]
        neg = H[i].sum(0) - pos
        a, pr = _hist_auc(pos, neg)
        ovr.append((a, pr, float(cls_w[i])))
    ovo = []
    for i in range(K - 1):
        for j in range(i + 1, K):
            a1, p1_ = _hist_auc(H[j, j], H[j, i])               # builder [i][j]: class j vs i by p_j
            a2, p2_ = _hist_auc(H[i, i], H[i, j])               # builder [j][i]: class i vs j by p_i
            a = (a1 + a2) / 2
            pr = (p1_ + p2_) / 2
            ovo.append((domain[i], domain[j], 0.0 if a != a else a, 0.0 if pr != pr else pr,
                        float(cls_w[i] + cls_w[j])))
    macro_ovr = float(np.mean([o[0] for o in ovr]))
    macro_ovr_pr = float(np.mean([o[1] for o in ovr]))
    pw = np.array([o[2] for o in ovr])
    weighted_ovr = float(np.sum([o[0] * o[2] for o in ovr]) / pw.sum()) if pw.sum() > 0 else float("nan")
    weighted_ovr_pr = float(np.sum([o[1] * o[2] for o in ovr]) / pw.sum()) if pw.sum() > 0 else float("nan")
    macro_ovo = float(np.mean([o[2] for o in ovo])) if ovo else float("nan")
    macro_ovo_pr = float(np.mean([o[3] for o in ovo])) if ovo else float("nan")
    ow = np.array([o[4] / n for o in ovo]) if ovo and n > 0 else np.zeros(0)
    weighted_ovo = float(np.sum([o[2] * q for o, q in zip(ovo, ow)]) / ow.sum()) if ow.sum() > 0 else float("nan")
    weighted_ovo_pr = float(np.sum([o[3] * q for o, q in zip(ovo, ow)]) / ow.sum()) if ow.sum() > 0 else \
        float("nan")
    pick = {"MACRO_OVR": (macro_ovr, macro_ovr_pr), "WEIGHTED_OVR": (weighted_ovr, weighted_ovr_pr),
            "MACRO_OVO": (macro_ovo, macro_ovo_pr), "WEIGHTED_OVO": (weighted_ovo, weighted_ovo_pr)}[t]

    def table(k):   # MultinomialAUC.getTable: OVR rows, macro/weighted OVR, OVO rows, macro/weighted OVO
        rows = [{"type": f"{domain[i]} vs Rest", "first_class_domain": domain[i], "second_class_domain": None,
                 "value": ovr[i][k]} for i in range(K)]
        rows += [{"type": "Macro OVR", "first_class_domain": None, "second_class_domain": None,
                  "value": macro_ovr if k == 0 else macro_ovr_pr},
                 {"type": "Weighted OVR", "first_class_domain": None, "second_class_domain": None,
                  "value": weighted_ovr if k == 0 else weighted_ovr_pr}]
        rows += [{"type": f"{o[0]} vs {o[1]}", "first_class_domain": o[0], "second_class_domain": o[1],
                  "value": o[2 + k]} for o in ovo]
        rows += [{"type": "Macro OVO", "first_class_domain": None, "second_class_domain": None,
                  "value": macro_ovo if k == 0 else macro_ovo_pr},
                 {"type": "Weighted OVO", "first_class_domain": None, "second_class_domain": None,
                  "value": weighted_ovo if k == 0 else weighted_ovo_pr}]
        return rows
    return {"AUC": pick[0], "pr_auc": pick[1], "auc_type": t, "multinomial_auc_table": table(0),
            "multinomial_aucpr_table": table(1)}


def multinomial_metrics(y_codes, probs, w=None, domain=None, hit_k=10, auc_type="AUTO", max_cm_size=None):
    """y_codes int64 [n] (-1 = NA), probs [n, K].  Every statistic is a sum
    (one bucketed all-reduce; the AUC histogram a second): no rows gathered."""
    ok = y_codes >= 0
    y, P = y_codes[ok].long(), probs[ok].to(torch.float64)
    w = torch.ones(y.numel(), dtype=torch.float64, device=y.device) if w is None else w[ok].to(torch.float64)
    K = P.shape[1]
    py = P[torch.arange(y.numel(), device=y.device), y].clamp(1e-15, 1)
    onehot = torch.nn.functional.one_hot(y, K).to(torch.float64)
    pred = torch.argmax(P, 1)
    cmat = torch.zeros((K, K), dtype=torch.float64, device=y.device)
    _ia(cmat.view(-1), y * K + pred, w)
    kk = min(hit_k, K)
    topk = torch.topk(P, kk, dim=1).indices
    hits = (topk == y.view(-1, 1)).to(torch.float64)
    hr_s = (torch.cumsum(hits, 1) * w.view(-1, 1)).sum(0)
    sums = torch.cat([torch.stack([w.sum(), -(w * torch.log(py)).sum(), (w * ((onehot - P) ** 2).sum(1)).sum(),
                                   torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device)]),
                      cmat.reshape(-1), hr_s])
    coll.allreduce_(sums)
    sh = sums.cpu().numpy()
    sw, ll_s, se_s, nobs = sh[:4]
    cm = sh[4:4 + K * K].reshape(K, K)
    hr = sh[4 + K * K:] / sw if sw > 0 else sh[4 + K * K:]
    logloss = float(ll_s / sw) if sw > 0 else float("nan")
    mse = float(se_s / sw) if sw > 0 else float("nan")
    rows = cm.sum(1)
    errs = [1 - cm[i, i] / rows[i] if rows[i] > 0 else 0.0 for i in range(K)]
    present = [i for i in range(K) if rows[i] > 0]
    mpce = float(np.mean([errs[i] for i in present])) if present else float("nan")
    dom = domain or [str(i) for i in range(K)]
    # ConfusionMatrix: no table past max_confusion_matrix_size classes (ModelMetricsMultinomial)
    cm_out = None if (max_cm_size is not None and K > int(max_cm_size)) else \
        {"domain": dom, "matrix": cm.tolist(), "errors": errs,
         "total_error": 1 - float(np.trace(cm)) / max(cm.sum(), 1e-300)}
    m = ModelMetricsMultinomial(MSE=mse, RMSE=math.sqrt(mse), logloss=logloss, mean_per_class_error=mpce,
                                nobs=int(nobs), cm=cm_out,
                                hit_ratio_table=[{"k": i + 1, "hit_ratio": float(hr[i])} for i in range(kk)],
                                domain=dom, AUC=float("nan"), pr_auc=float("nan"), auc_type=_auc_type(auc_type))
    ma = multinomial_auc(y, P, w, dom, auc_type)
    if ma is not None:
        m._m.update(ma)
    return m


def clustering_metrics(X, centers, assign, w=None):
    X = X.to(torch.float64)
    C = centers.to(torch.float64)
    w = torch.ones(X.shape[0], dtype=torch.float64, device=X.device) if w is None else w.to(torch.float64)
    d = ((X - C[assign]) ** 2).sum(1) * w
    k = C.shape[0]
    from ..core.groupsum import group_sum
    ws = group_sum(assign, torch.stack([d, w], 1), k)
    within, sizes = ws[:, 0].contiguous(), ws[:, 1].contiguous()
    sw = w.sum()
    mean = (X * w.view(-1, 1)).sum(0)
    stats = torch.cat([within, sizes, sw.view(1), mean])
    coll.allreduce_(stats)
    within, sizes, sw, mean = stats[:k], stats[k:2 * k], stats[2 * k], stats[2 * k + 1:] / stats[2 * k]
    tot = ((X - mean) ** 2).sum(1) * w
    totss = coll.allreduce_scalar(float(tot.sum()))
    tw = float(within.sum())
    return ModelMetricsClustering(tot_withinss=tw, totss=totss, betweenss=totss - tw,
                                  withinss=within.cpu().tolist(), size=sizes.cpu().tolist(),
                                  nobs=int(float(sw)))


# ---- sklearn-style regression metric functions over single-column frames
# (h2o-py h2o/model/models/regression.py h2o_mean_absolute_error & co.)
def _pair(y_actual, y_predicted, weights=None):
    a = y_actual.vec(y_actual.names[0]).as_float(torch.float64) if hasattr(y_actual, "vec") else \
        torch.as_tensor(y_actual, dtype=torch.float64)
    p = y_predicted.vec(y_predicted.names[0]).as_float(torch.float64) if hasattr(y_predicted, "vec") else \
        torch.as_tensor(y_predicted, dtype=torch.float64, device=a.device)
    w = None
    if weights is not None:
        w = weights.vec(weights.names[0]).as_float(torch.float64) if hasattr(weights, "vec") else \
            torch.as_tensor(weights, dtype=torch.float64, device=a.device)
    ok = ~torch.isnan(a) & ~torch.isnan(p)
    return a[ok], p[ok], (torch.ones_like(a[ok]) if w is None else w[ok])


def h2o_mean_absolute_error(y_actual, y_predicted, weights=None):
    a, p, w = _pair(y_actual, y_predicted, weights)
    return _wsum(w * (a - p).abs()) / _wsum(w)


def h2o_mean_squared_error(y_actual, y_predicted, weights=None):
    a, p, w = _pair(y_actual, y_predicted, weights)
    return _wsum(w * (a - p) ** 2) / _wsum(w)


def h2o_median_absolute_error(y_actual, y_predicted):
    a, p, _ = _pair(y_actual, y_predicted)
    return float(torch.median((a - p).abs()))


def h2o_explained_variance_score(y_actual, y_predicted, weights=None):
    a, p, w = _pair(y_actual, y_predicted, weights)
    sw = _wsum(w)
    d = a - p
    md, ma = _wsum(w * d) / sw, _wsum(w * a) / sw
    vd, va = _wsum(w * (d - md) ** 2) / sw, _wsum(w * (a - ma) ** 2) / sw
    return 1.0 - vd / va if va > 0 else 0.0


def h2o_r2_score(y_actual, y_predicted, weights=None):
    a, p, w = _pair(y_actual, y_predicted, weights)
    sw = _wsum(w)
    ma = _wsum(w * a) / sw
    ss_res, ss_tot = _wsum(w * (a - p) ** 2), _wsum(w * (a - ma) ** 2)
    return 1.0 - ss_res / ss_tot if ss_tot > 0 else float("nan")

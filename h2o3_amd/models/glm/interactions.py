"""Pairwise interaction features for GLM (interactions / interaction_pairs).

Reference: hex/DataInfo.java interaction vecs (InteractionWrappedVec): the
reference expands interactions lazily per chunk; here they are materialized
as extra frame columns on the device before the design matrix is built:
  numeric x numeric      -> product column  "a_b"
  categorical x categorical -> categorical "a_b" with levels "la_lb"
                              (training combinations; unseen -> NA)
  categorical x numeric  -> one numeric column per level "a_b.level"
                              (level indicator times the numeric value)
The recipe is stored on the model and replayed on scoring frames.
"""
from __future__ import annotations

import itertools

import torch

from ...core.vec import T_ENUM, Vec


def interaction_pairs(x, interactions=None, pairs=None):
    out = []
    if interactions:
        cols = list(interactions)
        out += list(itertools.combinations(cols, 2))
    for pr in pairs or []:
        a, b = pr
        if (a, b) not in out and (b, a) not in out:
            out.append((a, b))
    return out


def build_recipe(frame, pairs):
    rec = []
    for a, b in pairs:
        va, vb = frame.vec(a), frame.vec(b)
        ea, eb = va.type == T_ENUM, vb.type == T_ENUM
        if ea and eb:
            da, db = va.domain, vb.domain
            code = va.data.long() * len(db) + vb.data.long()
            ok = (va.data >= 0) & (vb.data >= 0)
            uniq = torch.unique(code[ok]).tolist()
            from ...parallel import cloud
            if cloud.is_distributed():
                from ...parallel import collectives as coll
                uniq = sorted(set(sum(coll.all_gather_object(uniq), [])))
            levels = [f"{da[c // len(db)]}_{db[c % len(db)]}" for c in uniq]
            rec.append({"kind": "cc", "a": a, "b": b, "name": f"{a}_{b}", "levels": levels})
        elif ea or eb:
            c, nmr = (a, b) if ea else (b, a)
            dom = frame.vec(c).domain
            rec.append({"kind": "cn", "a": c, "b": nmr, "name": f"{a}_{b}", "levels": list(dom[1:])})
        else:
            rec.append({"kind": "nn", "a": a, "b": b, "name": f"{a}_{b}"})
    return rec


def apply_recipe(frame, rec):
    """Returns (augmented frame, list of new predictor names)."""
    from ...core.frame import H2OFrame
    vecs, names, new_x = list(frame._vecs), list(frame.names), []
    for r in rec:
        va, vb = frame.vec(r["a"]), frame.vec(r["b"])
        if r["kind"] == "nn":
            vecs.append(Vec(va.as_float(torch.float64) * vb.as_float(torch.float64), "real"))
            names.append(r["name"])
            new_x.append(r["name"])
        elif r["kind"] == "cc":
            da, db = va.domain, vb.domain
            idx = {lv: i for i, lv in enumerate(r["levels"])}
            lut = torch.full((max(len(da), 1) * max(len(db), 1),), -1, dtype=torch.int32)
            for i, x in enumerate(da):
                for j, y in enumerate(db):
                    k = idx.get(f"{x}_{y}")
                    if k is not None:
                        lut[i * len(db) + j] = k
            lut = lut.to(va.data.device)
            ok = (va.data >= 0) & (vb.data >= 0)
            code = (va.data.long().clamp(min=0) * len(db) + vb.data.long().clamp(min=0))
            codes = torch.where(ok, lut[code], torch.full_like(va.data, -1))
            vecs.append(Vec(codes.to(torch.int32), T_ENUM, r["levels"]))
            names.append(r["name"])
            new_x.append(r["name"])
        else:
            dom = va.domain
            x = torch.nan_to_num(vb.as_float(torch.float64))
            for lv in r["levels"]:
                k = dom.index(lv) if lv in dom else -99
                col = torch.where(va.data == k, x, torch.zeros_like(x))
                nm = f"{r['name']}.{lv}"
                vecs.append(Vec(col, "real"))
                names.append(nm)
                new_x.append(nm)
    return H2OFrame.from_vecs(vecs, names), new_x

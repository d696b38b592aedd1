"""More /3 and /99 routes of the reference REST API: model inspection
(Tree, Word2Vec, FeatureInteraction, Friedman-Popescu H, SignificantRules,
TargetEncoderTransform, MakeGLMModel), persistence (frame save/load, grid
export/import, recovery resume, model JSON), session / cloud utilities and
listings.  Reference handlers: hex/tree/TreeHandler.java,
hex/word2vec/Word2VecHandler (water/api/Word2VecSynonymsV3,
Word2VecTransformV3), hex/api/FeatureInteractionHandler,
FriedmansPopescusHHandler, SignificantRulesHandler,
ai/h2o/targetencoding/TargetEncoderHandler, hex/glm/MakeGLMModelHandler,
water/api/FramesHandler (save / load), GridsHandler (Grid.bin),
RecoveryHandler, ModelsHandler (json export), SessionPropertiesHandler,
PingHandler, TypeaheadHandler, LeaderboardsHandler.  Registered by
rest.create_app through its `route` decorator."""
from __future__ import annotations

import glob
import json as _json
import os
import time


def register(app, route, ctx):
    from ..core import dkv
    from ..core.frame import H2OFrame
    from . import schemas as S
    from .rest import _HTTPError, _frame, _model, _put_frame
    api = ctx["api"]
    session_props: dict = {}

    # ------------------------------------------------------------- trees
    @route("GET", "/3/Tree")
    def tree(p, r):
        """TreeHandler: one tree in breadth-first order; children are given
        by their breadth-first index, `levels[i]` are the categorical levels
        routed INTO node i by its parent's split."""
        m = _model(p.get("model"))
        if not hasattr(m, "get_tree"):
            raise _HTTPError(400, f"Model {m.model_id} is not a tree-based model")
        tn = int(p.get("tree_number", 0) or 0)
        tc = p.get("tree_class")
        K = m._n_tree_classes()
        dom = m._spec.response_domain
        if K > 1:
            if tc in (None, ""):
                raise _HTTPError(400, "tree_class is required for multinomial models")
            tci = dom.index(tc) if tc in (dom or []) else int(tc)
        elif K == 1 and m._spec.nclasses == 2 and tc not in (None, "") and tc not in dom:
            raise _HTTPError(400, f"tree_class {tc} not in the response domain")
        else:
            tci = None
        if tn < 0 or tn * max(K, 1) >= len(m._forest):
            raise _HTTPError(400, f"Invalid tree number: {tn}")
        t = m.get_tree(tn, tci)
        names = list(m._spec.x)
        order, pos = [0], {0: 0}
        for i in order:                                     # breadth-first positions
            if t.left[i] >= 0:
                for c in (t.left[i], t.right[i]):
                    pos[c] = len(order)
                    order.append(c)
        n = len(order)
        left, right, feats, thr, nas, preds, levels, desc = [], [], [], [], [], [], [None] * n, []
        for i in order:
            leaf = t.left[i] < 0
            left.append(-1 if leaf else pos[t.left[i]])
            right.append(-1 if leaf else pos[t.right[i]])
            preds.append(float(t.value[i]))
            if leaf:
                feats.append(None)
                thr.append("NaN")
                nas.append(None)
                desc.append(f"Leaf node, prediction {float(t.value[i])}")
                continue
            f = names[t.feat[i]]
            feats.append(f)
            nas.append("LEFT" if t.na_left[i] else "RIGHT")
            if t.is_cat[i] and t.cat_left[i] is not None:
                mask = list(t.cat_left[i])
                levels[pos[t.left[i]]] = [k for k, b in enumerate(mask) if b]
                levels[pos[t.right[i]]] = [k for k, b in enumerate(mask) if not b]
                thr.append("NaN")
                desc.append(f"Categorical split on {f}")
            else:
                thr.append(float(t.thr[i]))
                desc.append(f"Numerical split on {f} < {float(t.thr[i])}; NA goes {nas[-1]}")
        return {"__meta": S.meta("TreeV3", "Iced"), "model": S.key(m.model_id, "Model"), "tree_number": tn,
                "tree_class": tc, "plain_language_rules": p.get("plain_language_rules", "AUTO"),
                "left_children": left, "right_children": right, "root_node_id": 0, "thresholds": thr,
                "features": feats, "levels": levels, "nas": nas, "descriptions": desc, "predictions": preds,
                "tree_decision_path": None, "decision_paths": None}

    # ----------------------------------------------------- model utilities
    @route("GET", "/3/Word2VecSynonyms")
    def w2v_synonyms(p, r):
        m = _model(p.get("model"))
        syn = m.find_synonyms(p.get("word"), int(p.get("count", 20) or 20))
        return {"__meta": S.meta("Word2VecSynonymsV3", "Iced"), "model": S.key(m.model_id, "Model"),
                "word": p.get("word"), "count": len(syn), "synonyms": list(syn.keys()),
                "scores": [float(v) for v in syn.values()]}

    @route("GET", "/3/Word2VecTransform")
    def w2v_transform(p, r):
        m = _model(p.get("model"))
        fr = m.transform(_frame(p.get("words_frame"), "words_frame"), p.get("aggregate_method") or "NONE")
        fid = _put_frame(fr)
        return {"__meta": S.meta("Word2VecTransformV3", "Iced"), "model": S.key(m.model_id, "Model"),
                "vectors_frame": S.key(fid)}

    def _tables(objs, name):
        out = []
        for i, t in enumerate(objs if isinstance(objs, (list, tuple)) else [objs]):
            if hasattr(t, "columns"):
                out.append(S.twodim_from_df(getattr(t, "attrs", {}).get("table_header", f"{name} {i}"), t))
            else:
                out.append(t)
        return out

    @route("POST", "/3/FeatureInteraction")
    def feature_interaction(p, r):
        m = _model(p.get("model_id"))
        tabs = m.feature_interaction(int(p.get("max_interaction_depth", 100) or 100),
                                     int(p.get("max_tree_depth", 100) or 100),
                                     int(p.get("max_deepening", -1) if p.get("max_deepening") is not None else -1))
        return {"__meta": S.meta("FeatureInteractionV3", "Iced"), "model_id": S.key(m.model_id, "Model"),
                "feature_interaction": _tables(tabs, "Feature Interaction")}

    @route("POST", "/3/FriedmansPopescusH")
    def friedman_h(p, r):
        m = _model(p.get("model_id"))
        h = m.h(_frame(p.get("frame")), list(p.get("variables") or []))
        return {"__meta": S.meta("FriedmansPopescusHV3", "Iced"), "model_id": S.key(m.model_id, "Model"),
                "h": float(h)}

    @route("POST", "/3/SignificantRules")
    def significant_rules(p, r):
        m = _model(p.get("model_id"))
        ri = m.rule_importance()
        return {"__meta": S.meta("SignificantRulesV3", "Iced"), "model_id": S.key(m.model_id, "Model"),
                "significant_rules_table": _tables(ri, "Rule Importance")[0]}

    @route("GET", "/3/TargetEncoderTransform")
    def te_transform(p, r):
        m = _model(p.get("model"))
        kw = {k: p[k] for k in ("blending", "inflection_point", "smoothing", "noise") if p.get(k) is not None}
        out = m.transform(_frame(p.get("frame")), as_training=bool(p.get("as_training", False)), **kw)
        return S.key(_put_frame(out))

    @route("POST", "/3/MakeGLMModel")
    def make_glm(p, r):
        from ..models.glm.glm import H2OGeneralizedLinearEstimator
        m = _model(p.get("model"))
        coefs = dict(zip(list(p.get("names") or []), [float(b) for b in p.get("beta") or []]))
        nm = H2OGeneralizedLinearEstimator.makeGLMModel(m, coefs, float(p.get("threshold", 0.5) or 0.5))
        if p.get("dest"):
            nm.model_id = p["dest"]
        dkv.put(nm.model_id, nm)
        return S.model_v3(nm.model_id, nm)

    # ------------------------------------------------------- persistence
    def _job(dest, desc, kind="Frame"):
        return {"__meta": S.meta("JobV3", "Job"), **S.job_v3(key_name=f"{desc}_{dest}", dest=dest, dest_kind=kind,
                                                              description=desc)}

    @route("POST", "/3/Frames/{fid}/save")
    def frame_save(p, r, fid):
        api.save_frame(_frame(fid), p.get("dir"), force=bool(p.get("force", True)))
        return {"__meta": S.meta("FrameSaveV3", "Iced"), "frame_id": S.key(fid), "dir": p.get("dir"),
                "job": _job(fid, "Save frame")}

    @route("POST", "/3/Frames/load")
    def frame_load(p, r):
        fid = p.get("frame_id")
        fr = api.load_frame(fid, p.get("dir"), force=bool(p.get("force", True)))
        _put_frame(fr, fid)
        return {"__meta": S.meta("FrameLoadV3", "Iced"), "frame_id": S.key(fid), "dir": p.get("dir"),
                "job": _job(fid, "Load frame")}

    @route("POST", "/3/Grid.bin/{gid}/export")
    def grid_export(p, r, gid):
        g = dkv.get(gid)
        if g is None or not hasattr(g, "model_ids"):
            raise _HTTPError(404, f"grid {gid} not found")
        path = api.save_grid(p.get("grid_directory"), gid,
                             save_params_references=bool(p.get("save_params_references", False)),
                             export_cross_validation_predictions=bool(p.get("export_cross_validation_predictions",
                                                                            False)))
        return {"__meta": S.meta("GridExportV3", "Iced"), "grid_id": gid, "grid_directory": p.get("grid_directory"),
                "path": path}

    @route("POST", "/3/Grid.bin/import")
    def grid_import(p, r):
        g = api.load_grid(p.get("grid_path"), bool(p.get("load_params_references", False)))
        dkv.put(g.grid_id, g)
        for mid in g.model_ids:
            mm = g.get_model(mid) if hasattr(g, "get_model") else dkv.get(mid)
            if mm is not None:
                dkv.put(mid, mm)
        return S.key(g.grid_id, "Grid")

    @route("POST", "/3/Recovery/resume")
    def recovery_resume(p, r):
        out = api.resume(p.get("recovery_dir"))
        for obj in out if isinstance(out, (list, tuple)) else [out]:
            k = getattr(obj, "grid_id", None) or getattr(obj, "project_name", None)
            if k:
                dkv.put(k, obj)
        return {"__meta": S.meta("RecoveryV3", "Iced"), "recovery_dir": p.get("recovery_dir")}

    @route("GET", "/99/Models/{mid}/json")
    def model_json(p, r, mid):
        m = _model(mid)
        d = p.get("dir")
        if not d:
            raise _HTTPError(400, "dir is required")
        if os.path.exists(d) and not p.get("force", True):
            raise _HTTPError(400, f"File {d} already exists")
        with open(d, "w") as f:
            _json.dump(S.jsonable(S.model_v3(mid, m)), f)
        return {"__meta": S.meta("ModelExportV3", "Iced"), "model_id": S.key(mid, "Model"), "dir": d}

    # ---------------------------------------------------------- listings
    @route("GET", "/3/ModelBuilders")
    def builders(p, r):
        from .rest import _ALGOS
        return {"__meta": S.meta("ModelBuildersV3", "Iced"),
                "model_builders": {a: {"algo": a, "algo_full_name": n, "visibility": "Stable",
                                       "can_build": ["Binomial", "Multinomial", "Regression"]}
                                   for a, n in _ALGOS.items()}}

    @route("GET", "/99/Leaderboards")
    def leaderboards(p, r):
        names = [k for k in dkv.keys() if hasattr(type(dkv.get(k)), "leaderboard")]
        return {"__meta": S.meta("LeaderboardsV99", "Iced", 99),
                "leaderboards": [{"project_name": k} for k in names]}

    @route("GET", "/3/Frames/{fid}/columns")
    def frame_columns(p, r, fid):
        fr = _frame(fid)
        return {"__meta": S.meta("FramesV3", "Frames"), "frame_id": S.key(fid),
                "frames": [{"frame_id": S.key(fid), "columns": [{"label": n, "type": fr.vec(n).type}
                                                                  for n in fr.names]}]}

    @route("GET", "/3/Frames/{fid}/columns/{col}")
    def frame_column(p, r, fid, col):
        fr = _frame(fid)
        if col not in fr.names:
            raise _HTTPError(404, f"Column {col} not found in frame {fid}")
        return {"__meta": S.meta("FramesV3", "Frames"), "frame_id": S.key(fid),
                "frames": [S.frame_v3(fid, fr[[col]], 0, int(p.get("row_count", 10) or 10), 0, -1, -1)]}

    @route("GET", "/3/Frames/{fid}/columns/{col}/domain")
    def frame_column_domain(p, r, fid, col):
        fr = _frame(fid)
        v = fr.vec(col)
        return {"__meta": S.meta("FrameV3", "Frames"), "frame_id": S.key(fid),
                "domain": [list(v.domain) if v.domain is not None else None]}

    @route("GET", "/3/Metadata/schemas")
    def schemas_list(p, r):
        return {"__meta": S.meta("MetadataV3", "Iced"), "schemas": []}

    # ------------------------------------------------- session / cloud
    @route("GET", "/3/Ping")
    def ping(p, r):
        from ..parallel import cloud
        return {"__meta": S.meta("PingV3", "Iced"), "cloud_uptime_millis": int(ctx["uptime_ms"]()),
                "cloud_healthy": True, "nodes": [{"ip_port": "127.0.0.1:54321", "healthy": True,
                                                   "rank": k} for k in range(cloud.world())]}

    @route("GET", "/3/SessionProperties")
    def session_get(p, r):
        k = p.get("key")
        return {"__meta": S.meta("SessionPropertyV3", "Iced"), "session_key": p.get("session_key"), "key": k,
                "value": session_props.get((p.get("session_key"), k))}

    @route("POST", "/3/SessionProperties")
    def session_set(p, r):
        session_props[(p.get("session_key"), p.get("key"))] = p.get("value")
        return {"__meta": S.meta("SessionPropertyV3", "Iced"), "session_key": p.get("session_key"),
                "key": p.get("key"), "value": p.get("value")}

    @route("DELETE", "/3/InitID")
    def end_session(p, r):
        return {"__meta": S.meta("InitIDV3", "Iced"), "session_key": p.get("session_key"), "session_properties": []}

    @route("DELETE", "/3/Models")
    def models_delete(p, r):
        from ..models.base import H2OEstimator
        for k in list(dkv.keys()):
            if isinstance(dkv.get(k), H2OEstimator):
                dkv.remove(k)
        return {"__meta": S.meta("ModelsV3", "Models")}

    @route("GET", "/3/Typeahead/files")
    def typeahead(p, r):
        """File-path completion for import dialogs (TypeaheadHandler)."""
        src = p.get("src") or ""
        limit = int(p.get("limit", 1000) or 1000)
        matches = sorted(glob.glob(os.path.expanduser(src) + "*"))[:limit]
        return {"__meta": S.meta("TypeaheadV3", "Iced"), "src": src, "limit": limit,
                "matches": [m + ("/" if os.path.isdir(m) else "") for m in matches]}

    @route("POST", "/3/UnlockKeys")
    def unlock_keys(p, r):
        return {"__meta": S.meta("UnlockKeysV3", "Iced")}

    @route("POST", "/3/CloudLock")
    def cloud_lock(p, r):
        return {"__meta": S.meta("CloudLockV3", "Iced"), "reason": p.get("reason")}

    @route("GET", "/3/JStack")
    def jstack(p, r):
        """Stack traces of the serving process's threads (JStackHandler)."""
        import sys
        import threading
        import traceback
        names = {t.ident: t.name for t in threading.enumerate()}
        traces = [{"thread": names.get(tid, str(tid)), "trace": "".join(traceback.format_stack(fr))}
                  for tid, fr in sys._current_frames().items()]
        return {"__meta": S.meta("JStackV3", "Iced"), "traces": [{"node": "rank0", "time": int(time.time() * 1000),
                                                                 "thread_traces": [t["thread"] + "\n" + t["trace"]
                                                                                   for t in traces]}]}

    @route("POST", "/3/PersistS3")
    def persist_s3(p, r):
        api.set_s3_credentials(p.get("secret_key_id"), p.get("secret_access_key"), p.get("session_token"))
        return {"__meta": S.meta("PersistS3CredentialsV3", "Iced"), "secret_key_id": "****"}

    @route("DELETE", "/3/PersistS3")
    def persist_s3_remove(p, r):
        api.remove_s3_credentials()
        return {"__meta": S.meta("PersistS3CredentialsV3", "Iced")}

    @route("POST", "/3/ParseSVMLight")
    def parse_svmlight(p, r):
        """Parse uploaded SVMLight sources (h2o-py uploads scipy sparse
        matrices this way)."""
        from ..core import parse as P
        srcs = [s["name"] if isinstance(s, dict) else str(s) for s in (p.get("source_frames") or [])]
        files = ctx["uploads"].resolve(srcs)
        fr = P._import_svmlight(files, p.get("destination_frame"))
        fid = _put_frame(fr, p.get("destination_frame") or fr.frame_id)
        return {"__meta": S.meta("ParseSVMLightV3", "Iced"), "destination_frame": S.key(fid),
                "job": _job(fid, "ParseSVMLight")}

    @route("GET", "/3/FrameChunks/{fid}")
    def frame_chunks(p, r, fid):
        """One chunk per rank: each rank holds one contiguous row shard."""
        fr = _frame(fid)
        return {"__meta": S.meta("FrameChunksV3", "Iced"), "frame_id": S.key(fid),
                "chunks": [{"chunk_id": 0, "row_count": int(fr.nrows), "node_idx": 0}]}

    @route("POST", "/3/ModelBuilders/{algo}/model_id")
    def calc_model_id(p, r, algo):
        """ModelBuildersHandler.calcModelId: a fresh unique model key."""
        from .rest import _algo_cls
        _algo_cls(algo)
        return {"__meta": S.meta("ModelIdV3", "Iced"), "model_id": dkv.make_key(algo)}

    @route("GET", "/99/Rapids/help")
    def rapids_help(p, r):
        """RapidsHandler.genHelp: the primitive names the interpreter knows."""
        from ..core.rapids import PRIMS
        return {"__meta": S.meta("RapidsHelpV3", "Iced", 99),
                "syntax": [{"name": k, "pattern": f"({k} ...)", "description": ""} for k in sorted(PRIMS)]}

    @route("GET", "/99/Sample")
    def sample(p, r):
        """The reference's example experimental endpoint: cloud status."""
        from ..parallel import cloud
        return S.cloud_v3(cloud.info(), time.time() - ctx["uptime_ms"]() / 1000)

    # ------------------------------------------------------- assembly
    assemblies: dict = {}

    @route("POST", "/99/Assembly")
    def assembly(p, r):
        """AssemblyHandler: the client's munging steps, each
        "name__Class__<Rapids AST over the frame 'dummy'>__inplace__newcols",
        applied in order (water/rapids/Assembly.java, transforms/*)."""
        import ast as _ast
        import re
        from ..core.rapids import rapids
        from .spmd import rand_hex
        steps = p.get("steps") or []
        if isinstance(steps, str):
            steps = _ast.literal_eval(steps)
        fr = _frame(p.get("frame"), "frame")
        cur = fr
        done = []
        for st in steps:
            name, cls, expr, inplace, newcols = st.split("__", 4) if st.count("__") >= 4 else (st, "", "", "", "")
            tmp = f"_asm_{rand_hex(12)}"
            dkv.put(tmp, cur)
            try:
                res = rapids(re.sub(r"\bdummy\b", tmp, expr))
            finally:
                dkv.remove(tmp)
            if cls == "H2OColSelect":
                cur = res
            else:
                m = re.search(r"cols_py\s+dummy\s+'([^']+)'", expr) or re.search(r'cols_py\s+dummy\s+"([^"]+)"', expr)
                col = m.group(1) if m else None
                if str(inplace).lower() == "true" and col is not None:
                    cur = cur.deep_copy(f"{fr.frame_id}_asm") if cur is fr else cur
                    cur[col] = res
                else:
                    names = [n for n in newcols.split("|") if n]
                    if names and len(names) == res.ncol:
                        res.names = names
                    cur = cur.cbind(res)
            done.append((name, cls))
        aid = f"Assembly_{rand_hex(16)}"
        assemblies[aid] = {"steps": done, "frame": fr.frame_id}
        rid = _put_frame(cur, f"{aid}_result")
        return {"__meta": S.meta("AssemblyV99", "Iced", 99), "assembly": S.key(aid, "Assembly"),
                "result": S.key(rid), "steps": steps, "frame": S.key(fr.frame_id)}

    @route("GET", "/99/Assembly.java/{aid}/{pojo_name}")
    def assembly_java(p, r, aid, pojo_name):
        from fastapi.responses import PlainTextResponse
        a = assemblies.get(aid)
        if a is None:
            raise _HTTPError(404, f"assembly {aid} not found")
        lines = ["import hex.genmodel.GenMunger;", "import hex.genmodel.easy.RowData;", "",
                 f"public class {pojo_name} extends GenMunger {{", f"  public {pojo_name}() {{",
                 f"    _steps = new Step[{len(a['steps'])}];"]
        lines += [f"    // step {i}: {n} ({c})" for i, (n, c) in enumerate(a["steps"])]
        lines += ["  }", "}"]
        return PlainTextResponse("\n".join(lines) + "\n")

    # ------------------------------------------------ frame utilities
    def _col(fr, spec):
        if isinstance(spec, dict):
            spec = spec.get("column_name")
        return spec

    @route("POST", "/99/Tabulate")
    def tabulate(p, r):
        """TabulateHandler: counts and mean response over a binned predictor
        (nbins_predictor) x binned response (nbins_response) grid."""
        import numpy as np
        fr = _frame(p.get("dataset"), "dataset")
        pc, rc, wc = _col(fr, p.get("predictor")), _col(fr, p.get("response")), _col(fr, p.get("weight"))
        cols = [c for c in (pc, rc, wc) if c]
        df = fr[cols].as_data_frame()
        nbp, nbr = int(p.get("nbins_predictor", 20) or 20), int(p.get("nbins_response", 10) or 10)
        w = df[wc].to_numpy(float) if wc else np.ones(len(df))

        def binned(v, nb):
            if v.dtype == object or str(v.dtype) == "category":
                lab = v.astype(str).to_numpy()
                levels = sorted(set(lab))
                return np.array([levels.index(x) for x in lab]), levels
            x = v.to_numpy(float)
            lo, hi = np.nanmin(x), np.nanmax(x)
            k = np.clip(((x - lo) / ((hi - lo) or 1) * nb).astype(int), 0, nb - 1)
            return k, [float(lo + (hi - lo) * i / nb) for i in range(nb)]
        bp, lp = binned(df[pc], nbp)
        br, lr = binned(df[rc], nbr)
        cnt = np.zeros((len(lp), len(lr)))
        np.add.at(cnt, (bp, br), w)
        resp = df[rc].to_numpy(float) if df[rc].dtype != object else br.astype(float)
        rs = np.zeros(len(lp))
        ws = np.zeros(len(lp))
        np.add.at(rs, bp, resp * w)
        np.add.at(ws, bp, w)
        ct = S.twodim("(Weighted) co-occurrence counts of '" + pc + "' and '" + rc + "'",
                      {pc: [str(x) for x in np.repeat(lp, len(lr))], rc: [str(x) for x in np.tile(lr, len(lp))],
                       "counts": cnt.reshape(-1).tolist()})
        rt = S.twodim("Mean value of '" + rc + "' and (weighted) counts",
                      {pc: [str(x) for x in lp], "mean " + rc: (rs / np.maximum(ws, 1e-300)).tolist(),
                       "counts": ws.tolist()})
        return {"__meta": S.meta("TabulateV3", "Iced"), "dataset": S.key(fr.frame_id), "count_table": ct,
                "response_table": rt}

    @route("POST", "/3/DataInfoFrame")
    def data_info_frame(p, r):
        """The model matrix of a frame (DataInfo expansion: one-hot
        categoricals, optionally standardized numerics)."""
        import torch
        from ..core.vec import T_REAL, Vec
        from ..models.datainfo import DataInfo
        fr = _frame(p.get("frame"), "frame")
        di = DataInfo(fr, list(fr.names), standardize=bool(p.get("standardize", False)),
                      use_all_factor_levels=bool(p.get("use_all", False)), pad_to=None)
        X, _ = di.expand(fr, dtype=torch.float64, pad=False)
        out = H2OFrame.from_vecs([Vec(X[:, j].contiguous(), T_REAL) for j in range(di.P)], list(di.coef_names))
        fid = _put_frame(out, f"{fr.frame_id}_datainfo")
        return {"__meta": S.meta("DataInfoFrameV3", "Iced"), "frame": S.key(fr.frame_id), "result": S.key(fid)}

    @route("GET", "/3/ComputeGram")
    def compute_gram(p, r):
        """GramHandler: X'WX of the expanded frame as a frame."""
        import torch
        from ..core.vec import T_REAL, Vec
        from ..models.datainfo import DataInfo
        fr = _frame(p.get("X"), "X")
        wc = _col(fr, p.get("W"))
        x = [c for c in fr.names if c != wc]
        di = DataInfo(fr, x, standardize=bool(p.get("standardize", False)),
                      use_all_factor_levels=bool(p.get("use_all_factor_levels", False)), pad_to=None)
        X, ok = di.expand(fr, dtype=torch.float64, pad=False)
        if bool(p.get("skip_missing", False)):
            X = X[ok]
        w = fr.vec(wc).as_float(torch.float64) if wc else None
        if w is not None and bool(p.get("skip_missing", False)):
            w = w[ok]
        G = X.T @ (X * w.view(-1, 1) if w is not None else X)
        from ..parallel import collectives as coll
        coll.allreduce_(G)
        out = H2OFrame.from_vecs([Vec(G[:, j].contiguous(), T_REAL) for j in range(G.shape[1])],
                                 list(di.coef_names))
        fid = _put_frame(out, p.get("destination_frame") or f"{fr.frame_id}_gram")
        return {"__meta": S.meta("GramV3", "Iced"), "X": S.key(fr.frame_id), "destination_frame": S.key(fid)}

    @route("POST", "/99/DCTTransformer")
    def dct(p, r):
        """DCTTransformerHandler: per-row orthonormal DCT-II (inverse: DCT-III)
        over the row reshaped to dimensions [x, y, z]."""
        import numpy as np
        import scipy.fft as sfft
        import torch
        from ..core.vec import T_REAL, Vec
        fr = _frame(p.get("dataset"), "dataset")
        dims = [int(d) for d in (p.get("dimensions") or [fr.ncol, 1, 1])]
        if int(np.prod(dims)) != fr.ncol:
            raise _HTTPError(400, f"dimensions {dims} do not match the {fr.ncol} columns")
        A = np.stack([fr.vec(c).as_float(torch.float64).cpu().numpy() for c in fr.names], 1)
        B = A.reshape((-1, *dims))
        axes = tuple(1 + i for i, d in enumerate(dims) if d > 1)
        f = sfft.idctn if p.get("inverse") else sfft.dctn
        Y = f(B, type=2, axes=axes, norm="ortho").reshape(A.shape)
        dev = fr.vec(fr.names[0]).data.device
        out = H2OFrame.from_vecs([Vec(torch.as_tensor(Y[:, j], device=dev).contiguous(), T_REAL)
                                  for j in range(Y.shape[1])], list(fr.names))
        fid = _put_frame(out, p.get("destination_frame") or f"{fr.frame_id}_dct")
        return {"__meta": S.meta("DCTTransformerV3", "Iced"), "dataset": S.key(fr.frame_id),
                "destination_frame": S.key(fid), "job": _job(fid, "DCT")}

    @route("GET", "/3/Find")
    def find(p, r):
        """FindHandler: previous / next row (from `row`) whose column value
        matches `match` (-1 when none)."""
        import numpy as np
        kv = p.get("key")
        fr = _frame(kv["name"] if isinstance(kv, dict) else kv, "key")
        row = int(p.get("row", 0) or 0)
        cols = [p["column"]] if p.get("column") else list(fr.names)
        hit = np.zeros(fr.nrows, dtype=bool)
        df = fr[cols].as_data_frame()
        m = str(p.get("match"))
        for c in cols:
            v = df[c]
            hit |= (v.astype(str).to_numpy() == m) | (v.isna().to_numpy() & (m in ("NA", "nan", "")))
        idx = np.nonzero(hit)[0]
        prev = idx[idx < row]
        nxt = idx[idx > row]
        return {"__meta": S.meta("FindV3", "Iced"), "column": p.get("column"), "row": row, "match": m,
                "prev": int(prev[-1]) if len(prev) else -1, "next": int(nxt[0]) if len(nxt) else -1}

    @route("GET", "/3/Frames/{fid}/export/{path}/overwrite/{force}")
    def frame_export_get(p, r, fid, path, force):
        from ..core.parse import export_file
        export_file(_frame(fid), path, force=str(force).lower() in ("true", "1"))
        return {"__meta": S.meta("FramesV3", "Frames"), "frame_id": S.key(fid), "path": path,
                "job": _job(fid, "Export")}

    @route("GET", "/3/Models.java/{mid}/preview")
    def pojo_preview(p, r, mid):
        from fastapi.responses import PlainTextResponse
        from ..mojo.pojo import to_java
        src = to_java(_model(mid))
        return PlainTextResponse("\n".join(src.splitlines()[:1000]))

    # ---------------------------------------------------- ModelMetrics
    def _all_metrics(mid=None, fid=None):
        from ..models.base import H2OEstimator
        out = []
        for k in list(dkv.keys()):
            m = dkv.get(k)
            if not isinstance(m, H2OEstimator) or (mid and k != mid):
                continue
            tf = getattr(getattr(m, "_spec", None), "frame", None)
            for mm in (m._training_metrics, m._validation_metrics):
                if mm is None:
                    continue
                if fid and getattr(tf, "frame_id", None) != fid:
                    continue
                out.append(S.metrics_v3(mm, m, getattr(tf, "frame_id", None)))
        return out

    @route("GET", "/3/ModelMetrics")
    def mm_all(p, r):
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"), "model_metrics": _all_metrics()}

    @route("GET", "/3/ModelMetrics/models/{mid}")
    def mm_model(p, r, mid):
        _model(mid)
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"), "model_metrics": _all_metrics(mid=mid)}

    @route("GET", "/3/ModelMetrics/frames/{fid}")
    def mm_frame(p, r, fid):
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"), "model_metrics": _all_metrics(fid=fid)}

    @route("GET", "/3/ModelMetrics/frames/{fid}/models/{mid}")
    def mm_frame_model(p, r, fid, mid):
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"),
                "model_metrics": _all_metrics(mid=mid, fid=fid)}

    for pth in ("/3/ModelMetrics", "/3/ModelMetrics/models/{mid}", "/3/ModelMetrics/frames/{fid}",
                "/3/ModelMetrics/frames/{fid}/models/{mid}", "/3/ModelMetrics/models/{mid}/frames/{fid}"):
        # metrics are computed on demand here, nothing is cached to delete
        route("DELETE", pth)(lambda p, r, **kw: {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"),
                                                 "model_metrics": []})

    # ------------------------------------------------------- monitoring
    @route("GET", "/3/WaterMeterCpuTicks/{node}")
    def cpu_ticks(p, r, node):
        """Per-core (user, system, other, idle) ticks of this node."""
        import psutil
        ticks = [[int(c.user * 100), int(c.system * 100), int((c.nice + getattr(c, "iowait", 0)) * 100),
                  int(c.idle * 100)] for c in psutil.cpu_times(percpu=True)]
        return {"__meta": S.meta("WaterMeterCpuTicksV3", "Iced"), "nodeidx": int(node), "cpu_ticks": ticks}

    @route("GET", "/3/WaterMeterIo")
    def io_meter(p, r):
        import psutil
        d = psutil.disk_io_counters()
        return {"__meta": S.meta("WaterMeterIoV3", "Iced"), "nodeidx": -1,
                "persist_stats": [{"backend": "local", "store_count": int(d.write_count) if d else 0,
                                   "store_bytes": int(d.write_bytes) if d else 0,
                                   "load_count": int(d.read_count) if d else 0,
                                   "load_bytes": int(d.read_bytes) if d else 0}]}

    route("GET", "/3/WaterMeterIo/{node}")(lambda p, r, node: io_meter(p, r))

    @route("GET", "/3/SteamMetrics")
    def steam_metrics(p, r):
        return {"__meta": S.meta("SteamMetricsV3", "Iced"), "version": 0,
                "idle_millis": int(time.time() * 1000 - ctx.get("last_request_ms", time.time() * 1000))}

    @route("GET", "/3/Profiler")
    def profiler(p, r):
        """Stack-trace sampling of the serving process (ProfilerHandler)."""
        import collections
        import sys
        import traceback
        depth = int(p.get("depth", 10) or 10)
        cnt = collections.Counter()
        for _ in range(10):
            for fr_ in sys._current_frames().values():
                cnt["".join(traceback.format_stack(fr_)[-depth:])] += 1
            time.sleep(0.005)
        return {"__meta": S.meta("ProfilerV3", "Iced"), "depth": depth,
                "nodes": [{"node_name": "rank0", "timestamp": int(time.time() * 1000),
                           "entries": [{"stacktrace": k, "count": v} for k, v in cnt.most_common()]}]}

    @route("POST", "/3/KillMinus3")
    def kill_minus3(p, r):
        """Thread dump to the log (the reference's kill -3)."""
        from ..utils import log
        log.info("KillMinus3 thread dump:\n" + "\n".join(jstack(p, r)["traces"][0]["thread_traces"]))
        return {"__meta": S.meta("KillMinus3V3", "Iced")}

    route("GET", "/3/KillMinus3")(kill_minus3)

    @route("GET", "/3/Metadata/schemaclasses/{cls}")
    def schema_class(p, r, cls):
        return {"__meta": S.meta("MetadataV3", "Iced"), "schemas": [{"name": cls, "fields": []}]}

    @route("GET", "/3/Metadata/endpoints/{path}")
    def endpoint_meta(p, r, path):
        routes = [{"__meta": S.meta("RouteV3", "Iced"), "url_pattern": rt.path, "http_method": next(iter(rt.methods))}
                  for rt in app.routes if hasattr(rt, "methods") and path in rt.path]
        return {"__meta": S.meta("MetadataV3", "Iced"), "routes": routes, "schemas": []}

    return app

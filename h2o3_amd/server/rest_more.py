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
        names = [k for k in dkv.keys() if hasattr(dkv.get(k), "leaderboard")]
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

    return app

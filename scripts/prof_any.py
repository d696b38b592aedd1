"""cProfile of one estimator's training on algo_survey2's 1M-row GPU frame
(ALGO = coxph | isolationforest | extendedisolationforest | glrm | infogram):
top functions by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ROWS", "1000000")
sys.argv = sys.argv[:1]
import importlib.util  # noqa: E402

spec = importlib.util.spec_from_file_location("s2", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                 "algo_survey2.py"))
src = open(spec.origin).read()
src = src[:src.index("cases = [")]          # the frame builders only
ns = {"__file__": spec.origin, "__name__": "s2"}
exec(compile(src, spec.origin, "exec"), ns)
E, fr, xs = ns["E"], ns["fr"], ns["xs"]
algo = os.environ.get("ALGO", "coxph")
mk = {"coxph": (lambda: E.H2OCoxProportionalHazardsEstimator(stop_column="time"), dict(x=xs[:10], y="y")),
      "isolationforest": (lambda: E.H2OIsolationForestEstimator(seed=1), dict(x=xs)),
      "extendedisolationforest": (lambda: E.H2OExtendedIsolationForestEstimator(seed=1), dict(x=xs)),
      "glrm": (lambda: E.H2OGeneralizedLowRankEstimator(k=5, seed=1, max_iterations=50), dict(x=xs))}[algo]
m = mk[0]()
m.train(training_frame=fr, **mk[1])      # warm-up (library loads, first-call costs)
m = mk[0]()
pr = cProfile.Profile()
t0 = time.time()
pr.enable()
m.train(training_frame=fr, **mk[1])
torch.cuda.synchronize()
pr.disable()
print(f"{algo} train_s {time.time() - t0:.2f}", flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)

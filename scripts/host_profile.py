"""cProfile of the GBM driver's host side (small N so device time is tiny)."""
import cProfile
import os
import pstats
import sys

sys.argv = ["bench.py", "--rows", os.environ.get("ROWS", "1000000"), "--steps", "20", "--warmup", "2"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
bench.main()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats("engine.py|tree_ops.py|gbm.py|collectives", 30)

"""Statistical line sampler of TreeGrower.grow (host-side hotspots); BENCH_ARGS = bench.py args."""
import sys, threading, time, collections
import os; sys.argv=['bench.py']+os.environ.get('BENCH_ARGS','--algo drf --rows 300000 --cols 60 --cat-cols 10 --cat-card 100 --steps 2 --warmup 0').split()
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import bench
main_id = threading.get_ident()
sys.setswitchinterval(0.0001)
cnt2 = collections.Counter()
cnt = collections.Counter()
stop = False
def sampler():
    while not stop:
        f = sys._current_frames().get(main_id)
        # find the innermost frame inside engine.py grow
        inner = None
        g_ = f
        while g_ is not None:
            if '/h2o3_amd/' in g_.f_code.co_filename:
                inner = g_
                break
            g_ = g_.f_back
        if inner is not None:
            cnt2[(inner.f_code.co_filename.split('/h2o3_amd/')[1], inner.f_code.co_name, inner.f_lineno)] += 1
        while f is not None:
            if f.f_code.co_name in ('grow', '_grow') and f.f_code.co_filename.endswith('engine.py'):
                cnt[f.f_lineno] += 1
                break
            f = f.f_back
        time.sleep(0.0005)
t = threading.Thread(target=sampler, daemon=True); t.start()
bench.main()
stop = True
t.join()
tot = sum(cnt.values())
src = open(os.environ.get('GRAFT_REPO_ROOT', '/root/repo') + '/h2o3_amd/models/tree/engine.py').read().splitlines()
for ln, c in cnt.most_common(25):
    print(f"{c:6d} {100*c/tot:5.1f}% L{ln}: {src[ln-1].strip()[:100]}")

tot2 = sum(cnt2.values())
print("innermost framework frames:")
for (fn, name, ln), c in cnt2.most_common(30):
    print(f"{c:6d} {100*c/tot2:5.1f}% {fn}:{ln} {name}")

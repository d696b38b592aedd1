"""Compact summary of a rocprofv3 --kernel-trace run: per-kernel totals and
the GPU busy / idle split of the timed window (the last `--steps` trees are
taken as the span between the first and last kernel of the tail of the trace).

usage: python scripts/prof_summary.py <trace.csv> <out.txt> [--after-gap-ms MS] [--per N]
--after-gap-ms: keep only the kernels after the last idle gap longer than MS
(the traced script sleeps between its warm-up and its timed trees);
--per: also report totals divided by N (e.g. per tree).
"""
import csv
import sys
from collections import defaultdict


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = []
    with open(src) as f:
        for r in csv.DictReader(f):
            try:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
            except (KeyError, ValueError):
                continue
    rows.sort()
    args = sys.argv[3:]
    gap_ms = float(args[args.index("--after-gap-ms") + 1]) if "--after-gap-ms" in args else None
    nper = int(args[args.index("--per") + 1]) if "--per" in args else 1
    if gap_ms is not None and rows:
        end_so_far, cut = rows[0][1], 0
        for i in range(1, len(rows)):
            if rows[i][0] - end_so_far > gap_ms * 1e6:
                cut = i
            end_so_far = max(end_so_far, rows[i][1])
        rows = rows[cut:]
    per = defaultdict(lambda: [0, 0])
    for s, e, k in rows:
        per[k][0] += 1
        per[k][1] += e - s
    # busy time = union of kernel intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0] if rows else 0
    with open(dst, "w") as out:
        out.write(f"kernels {len(rows)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
                  f"idle {(span - busy) / 1e6:.3f} ms ({100.0 * (span - busy) / max(span, 1):.1f}%)\n")
        if nper > 1:
            out.write(f"per unit (/{nper}): span {span / 1e6 / nper:.3f} ms  busy {busy / 1e6 / nper:.3f} ms  "
                      f"kernels {len(rows) / nper:.1f}\n")
        out.write(f"{'calls':>8} {'total_ms':>10} {'avg_us':>9} {'ms/unit':>8}  kernel\n")
        for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
            out.write(f"{c:8d} {t / 1e6:10.3f} {t / 1e3 / c:9.2f} {t / 1e6 / nper:8.3f}  {k[:110]}\n")


if __name__ == "__main__":
    main()

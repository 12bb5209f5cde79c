"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv): per-kernel-name
totals, busy time (union of kernel intervals) vs wall span, per step.
usage: trace_summary.py TRACE.csv STEPS [TOP]"""
import collections
import csv
import sys


def main(path, steps, top=25, marker=None, last=0):
    """marker / last: only the last `last` complete steps, a step starting at
    each launch whose name contains `marker` (once per step, e.g. k_prep_nctv
    of the train forward): steady state, without the first steps' set-up
    (model init, workspaces, lazy optimizer state)."""
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "0"))
                for r in rows)
    if marker and last:
        starts = [i for i, (_, _, k, _) in enumerate(iv) if marker in k]
        if len(starts) > last:
            iv = iv[starts[-last - 1]:starts[-1]]
            steps = last
    tot = collections.defaultdict(lambda: [0, 0])
    for s, e, k, _ in iv:
        t = tot[k.replace("(anonymous namespace)::", "").split("(")[0][-70:]]
        t[0] += e - s
        t[1] += 1
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    ksum = sum(v[0] for v in tot.values())
    print(f"launches/step {len(iv) / steps:.0f}  kernel-sum/step {ksum / steps / 1e3:.1f} us  "
          f"busy/step {busy / steps / 1e3:.1f} us  span/step {span / steps / 1e3:.1f} us")
    for k, (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / steps / 1e3:9.1f} us/step {c / steps:6.1f}/step {t / c / 1e3:8.2f} us  {k}")
    # per hardware queue (the training backward's weight-gradient stream runs on its own)
    byq = collections.defaultdict(lambda: [0, 0])
    for s, e, _, q in iv:
        byq[q][0] += e - s
        byq[q][1] += 1
    if len(byq) > 1:
        for q, (t, c) in sorted(byq.items(), key=lambda kv: -kv[1][1]):
            qiv = sorted((s, e) for s, e, _, qq in iv if qq == q)
            busy_q, cs, ce = 0, None, None
            for s, e in qiv:
                if ce is None or s > ce:
                    if ce is not None:
                        busy_q += ce - cs
                    cs, ce = s, e
                else:
                    ce = max(ce, e)
            busy_q += ce - cs
            print(f"queue {q}: {c / steps:.0f} launches/step, kernel-sum {t / steps / 1e3:.1f} us/step, "
                  f"busy {busy_q / steps / 1e3:.1f} us/step, idle in span {(span - busy_q) / steps / 1e3:.1f} us/step")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("steps", type=int)
    ap.add_argument("top", type=int, nargs="?", default=25)
    ap.add_argument("--marker", default=None, help="substring of the launch that starts a step (once per step)")
    ap.add_argument("--last", type=int, default=0, help="summarise only the last N steps")
    a = ap.parse_args()
    main(a.trace, a.steps, a.top, a.marker, a.last)

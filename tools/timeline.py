"""Concurrency of a rocprofv3 --kernel-trace run: how many kernels overlap, each kernel's mean time,
grid and share of the kernel residency, and the residency summed per frame (a frame starts at
k_frame_start).  For the frames-in-flight analysis of small parts.

    python tools/timeline.py gpurun_out/tl/..._kernel_trace.csv [--skip 0.3]

--skip drops that fraction of the trace from the front (warm-up, other phases).
"""
import argparse
import collections
import csv
import re


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:30]
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid // max(wg, 1),
                     r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=float, default=0.3)
    ap.add_argument("--until", type=float, default=1.0)
    ap.add_argument("--last-frames", type=int, default=0,
                    help="window = the last N frames (from the N-th last k_frame_start on)")
    a = ap.parse_args()
    rows = load(a.csv)
    t_lo, t_hi = rows[0][0], max(r[1] for r in rows)
    span = t_hi - t_lo
    lo, hi = t_lo + a.skip * span, t_lo + a.until * span
    if a.last_frames:
        fs = [r[0] for r in rows if r[2] == "k_frame_start"]
        lo, hi = fs[-a.last_frames], t_hi
    rows = [r for r in rows if r[0] >= lo and r[1] <= hi]
    if not rows:
        print("no kernels in the window")
        return
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    ev = []
    for s, e, *_ in rows:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    hist = collections.Counter()
    cur, prev = 0, ev[0][0]
    for t, d in ev:
        hist[cur] += t - prev
        cur += d
        prev = t
    tot = sum(hist.values())
    print("window %.3f ms, %d kernels" % ((t1 - t0) / 1e6, len(rows)))
    print("concurrent kernels: " + "  ".join("%d:%.1f%%" % (k, 100.0 * v / tot) for k, v in sorted(hist.items())))
    mean_c = sum(k * v for k, v in hist.items()) / tot
    print("mean concurrency %.2f" % mean_c)
    per = collections.defaultdict(list)
    for s, e, n, g, q in rows:
        per[n].append((e - s, g))
    frames = max(1, len(per.get("k_frame_start", [])))
    busy = sum(e - s for s, e, *_ in rows)
    print("frames %d; kernel residency per frame %.1f us; wall per frame %.1f us"
          % (frames, busy / frames / 1e3, (t1 - t0) / frames / 1e3))
    print("%-22s %6s %10s %10s %8s %7s" % ("kernel", "calls", "mean us", "per frame", "blocks", "share"))
    for n, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        tt = sum(x[0] for x in v)
        blocks = collections.Counter(x[1] for x in v).most_common(1)[0][0]
        print("%-22s %6d %10.1f %10.1f %8d %6.1f%%" % (n, len(v), tt / len(v) / 1e3, tt / frames / 1e3, blocks,
                                                    100.0 * tt / busy))


if __name__ == "__main__":
    main()

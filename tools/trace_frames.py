"""Per-frame kernel timeline from a rocprofv3 --kernel-trace CSV: the last N frames (a frame starts
at k_frame_setup), each kernel's duration and the gaps between them.

    python tools/trace_frames.py gpurun_out/trace8/run_kernel_trace.csv [--frames 2]
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--frames", type=int, default=2)
    a = ap.parse_args()
    seq = []
    for r in csv.DictReader(open(a.csv)):
        m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
        seq.append((m.group(1) if m else r["Kernel_Name"][:30], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    seq.sort(key=lambda x: x[1])
    starts = [i for i, x in enumerate(seq) if x[0] in ("k_frame_setup", "k_frame_start")]
    for fi in starts[-a.frames - 1:-1]:
        j, t0, prev = fi, seq[fi][1], seq[fi][1]
        while True:
            n, s, e = seq[j]
            print("%-28s %9.1f us  gap %6.1f  at %8.1f" % (n, (e - s) / 1e3, (s - prev) / 1e3, (s - t0) / 1e3))
            prev = e
            j += 1
            if j >= len(seq) or seq[j][0] in ("k_frame_setup", "k_frame_start"):
                break
        print("frame: %.1f us" % ((prev - t0) / 1e3))


if __name__ == "__main__":
    main()

"""Frame timeline from a rocprofv3 --kernel-trace CSV: per frame (split at
k_fill), its span, the time kernels were busy, and the largest idle gaps with
the kernels on either side.

    python tools/timeline.py <run_kernel_trace.csv> [hip_api_trace.csv]
"""
import csv
import sys
from collections import Counter


def short(n):
    return n.split("(")[0].replace("void ", "")[:40]


def main(path, api=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], []
    for r in rows:
        if short(r["Kernel_Name"]).startswith("k_fill") and cur:
            frames.append(cur)
            cur = []
        cur.append(r)
    frames.append(cur)
    for fi, fr in enumerate(frames):
        t0, t1 = int(fr[0]["Start_Timestamp"]), int(fr[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in fr)
        gaps = []
        for a, b in zip(fr, fr[1:]):
            gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), short(a["Kernel_Name"]),
                         short(b["Kernel_Name"])))
        per = Counter()
        for g, a, b in gaps:
            per[(a, b)] += g
        print(f"frame {fi}: span {(t1 - t0) / 1e6:.2f} ms, kernels busy {busy / 1e6:.2f} ms, "
              f"{len(fr)} kernels, gap total {sum(g for g, _, _ in gaps) / 1e6:.2f} ms")
        for (a, b), g in per.most_common(6):
            print(f"    gaps {a} -> {b}: {g / 1e6:.2f} ms")
        gaps.sort(reverse=True)
        for g in gaps[:3]:
            print(f"    largest gap {g[0] / 1e3:.1f} us {g[1]} -> {g[2]}")
    if api:
        tot = Counter()
        cnt = Counter()
        for r in csv.DictReader(open(api)):
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            tot[r["Function"]] += d
            cnt[r["Function"]] += 1
        for f, d in tot.most_common(12):
            print(f"api {f}: {d / 1e6:.2f} ms over {cnt[f]} calls")


if __name__ == "__main__":
    main(*sys.argv[1:])

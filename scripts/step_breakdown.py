"""Per-step kernel-time breakdown from a rocprofv3 kernel trace of `bench.py` (one graph-replayed
denoising step = the 48 self-attention launches after the first 48, plus everything between them).

usage: python scripts/step_breakdown.py <run_kernel_trace.csv> [step_index]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    selfattn = [r for r in rows if "attn_fwd" in r["Kernel_Name"] and dur(r) > 5_000_000]
    blocks = 48
    if len(selfattn) < (step + 1) * blocks:
        sys.exit(f"trace holds {len(selfattn)} self-attention launches, step {step} needs {(step + 1) * blocks}")
    a = int(selfattn[step * blocks]["Start_Timestamp"])
    b = int(selfattn[(step + 1) * blocks - 1]["End_Timestamp"])
    ks = [r for r in rows if int(r["Start_Timestamp"]) >= a and int(r["End_Timestamp"]) <= b]
    agg, cnt = collections.Counter(), collections.Counter()
    busy, last = 0, a
    for r in ks:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += max(0, en - max(st, last))
        last = max(last, en)
        n = r["Kernel_Name"]
        if n.startswith(("Cijk", "Custom")):
            k = "hipBLASLt MT" + n.split("MT")[1].split("_")[0] + f" grid {r['Grid_Size_X']}"
        elif "attn_fwd" in n:
            k = ("attn_fwd_w4 self" if "attn_fwd_w4" in n else "attn_fwd_d128 self") if dur(r) > 5_000_000 \
                else ("attn_fwd_w4 cross" if "attn_fwd_w4" in n else "attn_fwd_d128 cross")
        else:
            k = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[k] += dur(r)
        cnt[k] += 1
    tot = sum(agg.values())
    print(f"step {step}: span {(b - a) / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms, {len(ks)} kernels")
    print(f"{'kernel':48s} {'ms/step':>9s} {'share':>6s} {'n':>4s} {'avg us':>8s}")
    for k, v in agg.most_common():
        print(f"{k:48s} {v / 1e6:9.1f} {100 * v / tot:5.1f}% {cnt[k]:4d} {v / cnt[k] / 1e3:8.0f}")


if __name__ == "__main__":
    main()

"""GPU busy fraction of a rocprofv3 kernel trace over a window: the union of kernel intervals divided
by the window's span, and the largest idle gaps -- to tell a GPU-bound step (busy ~100 %) from a
launch- or sync-bound one.
usage: python3 scripts/gpu_busy.py <run_kernel_trace.csv> [first_kernel_index] [last_kernel_index]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
    ks = rows[lo:hi]
    a, b = int(ks[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in ks)
    busy, last, gaps = 0, a, []
    for r in ks:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if st > last:
            gaps.append((st - last, r["Kernel_Name"][:60]))
        busy += max(0, en - max(st, last))
        last = max(last, en)
    print(f"{len(ks)} kernels, span {(b - a) / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({100.0 * busy / (b - a):.1f} %), "
          f"idle {(b - a - busy) / 1e6:.1f} ms in {len(gaps)} gaps")
    for g, n in sorted(gaps, reverse=True)[:8]:
        print(f"  gap {g / 1e3:8.1f} us before {n}")


if __name__ == "__main__":
    main()

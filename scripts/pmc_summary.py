"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_<which>/p*_counter_collection.csv) for the
named kernel: per-dispatch counter values averaged over dispatches of that kernel."""
import csv, glob, os, sys, collections
which, kname = sys.argv[1], sys.argv[2]
d = os.path.join("gpurun_out", f"pmc_{which}")
vals = collections.defaultdict(list)
dur = []
for f in sorted(glob.glob(os.path.join(d, "p*_counter_collection.csv"))):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]:
            continue
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (c, dsp), v in per.items():
        vals[c].append(v)
for f in sorted(glob.glob(os.path.join(d, "p*_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
ms = sorted(dur)[len(dur) // 2]
print(f"{kname}: median dispatch {ms:.3f} ms over {len(dur)} profiled dispatches")
for c in sorted(avg):
    print(f"  {c:28s} {avg[c]:.4g}")
if "GRBM_GUI_ACTIVE" in avg:
    print(f"  effective clock ~ {avg['GRBM_GUI_ACTIVE'] / 8 / (ms * 1e-3) / 1e9:.2f} GHz (GRBM/8/time)")
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if k in avg:
            print(f"  {k:28s} {100 * avg[k] / wc:5.1f} % of wave-cycles")
if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
    # MFMA busy cycles summed over SIMDs: utilisation = busy / (SIMDs * GPU cycles)
    gpu_cycles = avg["GRBM_GUI_ACTIVE"] / 8
    print(f"  MFMA busy / (1024 SIMDs x cycles) = {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * gpu_cycles):.3f}")
if len(dur) > 1 and "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
    # all dispatches together (kernels of many shapes, e.g. the VAE convs): time-weighted
    tot = sum(vals["GRBM_GUI_ACTIVE"]) / 8
    print(f"  all dispatches: MFMA busy {sum(vals['SQ_VALU_MFMA_BUSY_CYCLES']) / (1024 * tot):.3f}, "
          f"{sum(dur) / max(1, len(glob.glob(os.path.join(d, 'p*_kernel_trace.csv')))):.1f} ms per pass")
if "FETCH_SIZE" in avg:
    print(f"  HBM read  ~ {2 * avg['FETCH_SIZE'] * 1024 / 1e9:.3f} GB/dispatch (FETCH_SIZE x2 gfx950 correction)")
if "WRITE_SIZE" in avg:
    print(f"  HBM write ~ {avg['WRITE_SIZE'] * 1024 / 1e9:.3f} GB/dispatch")
if "TCC_HIT_sum" in avg:
    print(f"  L2 hit rate {avg['TCC_HIT_sum'] / (avg['TCC_HIT_sum'] + avg['TCC_MISS_sum']):.3f}")

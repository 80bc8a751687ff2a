"""Per kernel family of one benchmarked step (scripts/pmc_step.sh): total time, MFMA busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM cycles), effective clock (GRBM_GUI_ACTIVE / 8 / time),
SQ_WAIT_ANY share of wave cycles.  Usage: pmc_step_summary.py <dir>"""
import collections, csv, glob, os, sys

d = sys.argv[1]
fam = lambda n: ("attn_fwd_w4" if "attn_fwd_w4" in n else "attn_fwd_d128" if "attn_fwd_d128" in n
                 else "gemm_bf16_tn_4w" if "gemm_bf16_tn_4w" in n else "hipBLASLt" if n.startswith("Cijk")
                 else n.split("(")[0].split("<")[0][-40:])
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        vals[(r["Dispatch_Id"], r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
dur = {}
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for (disp, name), c in vals.items():
    a = agg[fam(name)]
    a["n"] += 1
    a["t"] += dur.get(disp, 0.0)
    for k, v in c.items():
        a[k] += v
print(f"{'kernel family':42s} {'ms':>8s} {'n':>5s} {'MFMA busy':>10s} {'clock GHz':>10s} {'wait %':>7s}")
for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["t"])[:12]:
    cyc = a["GRBM_GUI_ACTIVE"] / 8
    busy = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc) if cyc else 0
    clk = cyc / a["t"] / 1e9 if a["t"] else 0
    wait = 100 * a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"] if a["SQ_WAVE_CYCLES"] else 0
    print(f"{k:42s} {1e3 * a['t']:8.1f} {int(a['n']):5d} {busy:10.3f} {clk:10.2f} {wait:7.1f}")

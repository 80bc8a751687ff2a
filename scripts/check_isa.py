"""Build-time ISA guards of the hand-written GEMM kernels (run by `make` after gemm.o is built).

The 4-wave GEMMs (gemm_bf16_tn_4w, gemm_fp8_tn_4w) read their 256 accumulators with an inline-asm
v_accvgpr_read at the point of use (acc_rd, csrc/gemm.hip).  That is correct only while the compiler
makes no copy of an accumulator AGPR: an asm read right after a v_accvgpr_write the hazard
recognizer cannot pair returned stale values in r4 (profiles/r4/fp8_8b_path_debug.log).  So, per
instantiation that reads through acc_rd (every one but the fp8 8-B fallback, which reads plainly):
  * no v_accvgpr_write / v_accvgpr_mov at all (the accumulators are written by MFMAs only),
  * exactly 512 v_accvgpr_read (256 in the tile epilogue, 256 in the split-piece path),
  * no scratch (a spilled accumulator or fragment would be a scratch round trip in the K loop).
And the tile-queue atomic (W4Grab::issue) must be a single returning global atomic add per kernel
(the compiler's atomic optimizer off for gemm.o: Makefile).

usage: check_isa.py <gemm.o | libvstyler.so>   (exit 1 with the offending kernels listed)"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")


def code_objects(obj, d):
    """The gfx950 code objects of a host object or shared library: its .hip_fatbin section holds one
    offload bundle per linked translation unit (one for gemm.o, seven for libvstyler.so)."""
    fat = os.path.join(d, "fat.bin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", obj,
                    os.path.join(d, "copy.o")], check=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, a in enumerate(starts):
        part = os.path.join(d, f"b{i}.bin")
        with open(part, "wb") as f:
            f.write(data[a:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(d, f"dev{i}.co")
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        if os.path.getsize(co):
            out.append(co)
    return out


def kernels(co):
    text = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout
    out = {}
    for part in re.split(r"\n(?=[0-9a-f]+ <_Z)", text):
        m = re.match(r"[0-9a-f]+ <(_Z[^>]+)>:", part)
        if m:
            out[m.group(1)] = part
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    scratch, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
        if m and cur is not None:
            scratch[cur] = int(m.group(1))
        m = re.match(r"\s*-\s*\.agpr_count", line)
        if m:
            cur = None
    return out, scratch


def main():
    obj = sys.argv[1]
    bad = []
    ks, scratch = {}, {}
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(obj, d):
            k, sc = kernels(co)
            ks.update(k)
            scratch.update(sc)
    checked = 0
    for name, body in ks.items():
        if "_tn_4w" not in name:
            continue
        eight_b = "gemm_fp8_tn_4wILb0" in name          # the fp8 8-B fallback reads plainly
        nw = len(re.findall(r"\bv_accvgpr_write", body))
        nm = len(re.findall(r"\bv_accvgpr_mov", body))
        nr = len(re.findall(r"\bv_accvgpr_read", body))
        na = len(re.findall(r"\bglobal_atomic_add\b.*\bsc0\b", body))
        if not eight_b and (nw or nm or nr != 512):
            bad.append(f"{name}: accvgpr write {nw} mov {nm} read {nr} (want 0 / 0 / 512)")
        if scratch.get(name, 0) and not eight_b:
            bad.append(f"{name}: {scratch[name]} B of scratch")
        if na < 1:
            bad.append(f"{name}: no returning tile-queue atomic")
        checked += 1
    if checked < 13:
        bad.append(f"only {checked} gemm_*_4w kernels found (expected 13)")
    if bad:
        print("check_isa: FAILED\n  " + "\n  ".join(bad))
        sys.exit(1)
    print(f"check_isa: {checked} gemm_*_4w kernels OK (no accumulator AGPR copies, 512 acc_rd reads, no scratch)")


if __name__ == "__main__":
    main()

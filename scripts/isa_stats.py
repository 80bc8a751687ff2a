"""Register / scratch statistics and disassembly of the gfx950 code object of one csrc/*.hip file.

usage: python3 scripts/isa_stats.py <file.hip> [name-substring ...] [--dump out.s]
Compiles the file device-only (the Makefile's flags), unbundles the gfx950 code object and prints,
per kernel whose mangled name contains one of the substrings: VGPRs, AGPRs, SGPRs, spills and
private (scratch) bytes.  Build-time checks (scripts/check_isa.py) reuse `code_object()`."""
import os
import re
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LLVM = os.path.join(ROCM, "lib", "llvm", "bin")
CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-styler_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics"]
EXTRA = {"attention.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=max-ilp"],
         "attention_w4.hip": ["-fno-slp-vectorize"],
         "gemm.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}


def code_object(src, workdir):
    """Path of the unbundled gfx950 code object of csrc/<src> (compiled device-only into workdir)."""
    path = src if os.path.isabs(src) else os.path.join(CSRC, src)
    dev = os.path.join(workdir, "dev.o")
    co = os.path.join(workdir, "dev.co")
    subprocess.run([os.path.join(ROCM, "bin", "hipcc"), *FLAGS, *EXTRA.get(os.path.basename(path), []),
                    "--cuda-device-only", "-c", "-o", dev, path], check=True, stderr=subprocess.DEVNULL)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={dev}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def kernel_stats(co):
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "agpr_count":            # first key of a kernel's map (alphabetical order)
            cur = {}
            out.append(cur)
        if cur is not None:
            cur[key] = val
    return out


def disassemble(co):
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout


def main():
    args = [a for a in sys.argv[1:]]
    dump = None
    if "--dump" in args:
        i = args.index("--dump")
        dump = args[i + 1]
        del args[i:i + 2]
    src, subs = args[0], args[1:]
    with tempfile.TemporaryDirectory() as d:
        co = code_object(src, d)
        for k in kernel_stats(co):
            name = k.get("name", "?")
            if subs and not any(s in name for s in subs):
                continue
            print(f"vgpr {k.get('vgpr_count')} agpr {k.get('agpr_count')} sgpr {k.get('sgpr_count')} "
                  f"spill v/s {k.get('vgpr_spill_count')}/{k.get('sgpr_spill_count')} "
                  f"scratch {k.get('private_segment_fixed_size')} lds {k.get('group_segment_fixed_size')}  {name}")
        if dump:
            with open(dump, "w") as f:
                f.write(disassemble(co))


if __name__ == "__main__":
    main()

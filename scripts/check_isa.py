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
(the compiler's atomic optimizer off for gemm.o: Makefile), whose destination VGPR nothing touches
between the atomic and the `s_waitcnt vmcnt` + `v_readfirstlane` that consume it (queue_value_hazards;
also checked in the attention kernels, which take their items from the same kind of queue).
The VAE flash attention (vae_attn_kernel, three widths) must compile without scratch: its 192
accumulator registers per lane at C = 384 fit only while the compiler keeps them in AGPRs.

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


def _vregs(operands):
    """VGPR numbers named in an operand string (v7, v[4:7])."""
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", operands):
        out.update(range(int(a), int(b) + 1))
    out.update(int(r) for r in re.findall(r"\bv(\d+)\b", operands))
    return out


def _instructions(body):
    """(address, opcode, operands, branch target address or None) of a kernel's disassembly."""
    m = re.match(r"([0-9a-f]+) <", body)
    base = int(m.group(1), 16) if m else 0
    out = []
    for ln in body.splitlines():
        m = re.match(r"\s*([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", ln)
        if not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        t = re.search(r"<_Z[^>+]*\+0x([0-9a-f]+)>", ln)
        out.append((addr, op, args, base + int(t.group(1), 16) if t and op.startswith(("s_branch", "s_cbranch"))
                    else None))
    return out


def queue_value_hazards(body):
    """The tile-queue atomic (vs_queue_issue, csrc/common.h) returns its value in a VGPR the compiler
    believes ready when the asm ends; only vs_queue_value's `s_waitcnt vmcnt(W)` + `v_readfirstlane`
    wait for it.  A copy (or any other read, or a reuse) of that VGPR placed between the two by the
    register allocator would read a stale tile id.  For every such atomic (returning, EXEC set to
    lane 0 just before it), follow every control-flow path from it (branches taken and not taken) to
    the first v_readfirstlane of its destination VGPR, and report any instruction on the way that
    READS that VGPR, or a readfirstlane reached without a vmcnt wait after the atomic.
    A path that overwrites the VGPR or ends the program is one on which the allocator holds the value
    dead (paths correlated with the kernel's own `wave == 0` branches that it never takes); at least
    one path must consume it."""
    insts = _instructions(body)
    at = {addr: i for i, (addr, _, _, _) in enumerate(insts)}
    issues, n_atomics = [], 0
    stores = ("global_store", "buffer_store", "ds_write", "ds_store", "flat_store", "scratch_store")
    for i, (_, op, args, _) in enumerate(insts):
        # vs_queue_issue's atomic: returning (sc0), issued with EXEC = lane 0 by the asm itself
        if op != "global_atomic_add" or not re.search(r"\bsc0\b", args) or \
                not any(o == "s_mov_b64" and a.startswith("exec, 1") for _, o, a, _ in insts[max(0, i - 2):i]):
            continue
        n_atomics += 1
        dst = int(re.match(r"v(\d+)", args).group(1))
        consumed = False
        todo, seen = [(i + 1, False)], set()
        while todo:
            j, waited = todo.pop()
            while j < len(insts) and (j, waited) not in seen:
                seen.add((j, waited))
                _, op2, args2, tgt = insts[j]
                if op2 == "s_waitcnt" and "vmcnt" in args2:
                    waited = True
                if op2 == "v_readfirstlane_b32" and dst in _vregs(args2.split(",", 1)[1]):
                    consumed = True
                    if not waited:
                        issues.append(f"v{dst}: v_readfirstlane at {insts[j][0]:#x} with no vmcnt wait after the atomic")
                    break
                ops = args2.split(",", 1)
                read = _vregs(args2) if op2.startswith(stores) or (op2.startswith("global_atomic")
                                                                   and "sc0" not in args2) else \
                    (_vregs(ops[1]) if len(ops) > 1 else set())
                if dst in read:          # a copy / use of the value before it has landed
                    issues.append(f"v{dst}: '{op2} {args2}' at {insts[j][0]:#x} reads it between the atomic "
                                  f"and its vmcnt + readfirstlane")
                    break
                if dst in _vregs(ops[0]):    # overwritten: the value is dead on this path (the
                    break                    # allocator's view of a path the kernel never takes)
                if op2 == "s_endpgm":
                    break
                if tgt is not None:
                    if tgt not in at:
                        issues.append(f"v{dst}: branch to unknown address {tgt:#x}")
                        break
                    if op2 == "s_branch":
                        j = at[tgt]
                        continue
                    todo.append((at[tgt], waited))
                j += 1
        if not consumed:
            issues.append(f"v{dst}: never consumed by a v_readfirstlane on any path")
    return n_atomics, issues


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
        bad += [f"{name}: {msg}" for msg in queue_value_hazards(body)[1]]
        checked += 1
    if checked < 13:
        bad.append(f"only {checked} gemm_*_4w kernels found (expected 13)")
    nq = 0
    for name, body in ks.items():            # the attention kernels take items from the same queues
        if "attn_fwd_w4" in name:
            n, issues = queue_value_hazards(body)
            nq += n
            bad += [f"{name}: {msg}" for msg in issues]
    nv = 0
    for name, body in ks.items():            # the VAE flash attention: accumulators stay in AGPRs, no spill
        if "vae_attn_kernel" in name:
            nv += 1
            if scratch.get(name, 0):
                bad.append(f"{name}: {scratch[name]} B of scratch")
    if nv != 3:
        bad.append(f"{nv} vae_attn_kernel instances found (expected 3: C = 128, 256, 384)")
    if bad:
        print("check_isa: FAILED\n  " + "\n  ".join(bad))
        sys.exit(1)
    print(f"check_isa: {checked} gemm_*_4w kernels OK (no accumulator AGPR copies, 512 acc_rd reads, no scratch, "
          f"queue atomics consumed only behind their vmcnt wait; {nq} in the attention kernels; "
          f"{nv} VAE attention kernels without scratch)")


if __name__ == "__main__":
    main()

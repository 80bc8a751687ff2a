"""Private copy of the image's ROCm hipBLASLt for libvstyler (run by the csrc Makefile).

In a Python process torch has already loaded its own bundled hipBLASLt + rocRoller (the ROCm 7.0
builds) under the SONAMEs libhipblaslt.so.1 / librocroller.so.1, so the image's faster ROCm 7.2
build cannot be loaded next to them under those names: the dynamic loader would hand back torch's
copies.  This writes copies of /opt/rocm/lib/libhipblaslt.so.1 and librocroller.so.1 whose SONAMEs
(and hipBLASLt's NEEDED entry for rocRoller) are renamed in the .dynstr section, in place and with
names of the same length, so libvstyler can dlopen them as separate objects (csrc/blaslt.hip).
Nothing else in the files changes.

usage: python scripts/vendor_blaslt.py <out_dir> [rocm_lib_dir]
"""
import os
import shutil
import struct
import sys

RENAMES = {b"libhipblaslt.so.1": b"libvsblaslt7.so.1", b"librocroller.so.1": b"libvsroller7.so.1"}
FILES = {"libhipblaslt.so.1": "libvsblaslt7.so.1", "librocroller.so.1": "libvsroller7.so.1"}


def dynstr_range(data):
    """(offset, size) of the .dynstr section of an ELF64 little-endian file."""
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError("not an ELF64 LE file")
    e_shoff, = struct.unpack_from("<Q", data, 0x28)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sh(i):
        base = e_shoff + i * e_shentsize
        name, typ = struct.unpack_from("<II", data, base)
        off, size = struct.unpack_from("<QQ", data, base + 0x18)
        return name, typ, off, size
    _, _, stroff, _ = sh(e_shstrndx)
    for i in range(e_shnum):
        name, typ, off, size = sh(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".dynstr":
            return off, size
    raise ValueError("no .dynstr")


def patch(src, dst):
    data = bytearray(open(src, "rb").read())
    off, size = dynstr_range(data)
    n = 0
    for old, new in RENAMES.items():
        assert len(old) == len(new)
        pat = b"\0" + old + b"\0"
        i = data.find(pat, off, off + size)
        while i >= 0:
            data[i + 1:i + 1 + len(old)] = new
            n += 1
            i = data.find(pat, i + 1, off + size)
    tmp = dst + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    shutil.copymode(src, tmp)
    os.replace(tmp, dst)
    return n


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    out = argv[0]
    lib = argv[1] if len(argv) > 1 else os.path.join(os.environ.get("ROCM_PATH") or "/opt/rocm", "lib")
    os.makedirs(out, exist_ok=True)
    for src, dst in FILES.items():
        s, d = os.path.join(lib, src), os.path.join(out, dst)
        if not os.path.exists(s):
            print(f"vendor_blaslt: {s} missing; libvstyler keeps the link-time hipBLASLt")
            return
        if os.path.exists(d) and os.path.getmtime(d) >= os.path.getmtime(os.path.realpath(s)):
            continue
        n = patch(os.path.realpath(s), d)
        print(f"vendor_blaslt: {d} ({n} names renamed)")
    # the copy finds its kernel library at <its dir>/hipblaslt/library (dladdr): a link to the ROCm
    # tree (same path on the GPU box: same image), made here so libvstyler never writes at run time
    link = os.path.join(out, "hipblaslt")
    target = os.path.join(lib, "hipblaslt")
    if os.path.islink(link) and os.readlink(link) != target:
        os.remove(link)
    if not os.path.lexists(link):
        os.symlink(target, link)
        print(f"vendor_blaslt: {link} -> {target}")


if __name__ == "__main__":
    main()

"""A/B of the HBM-bound row kernels at the 14B 832x480x73 CFG shapes (M = 59280 rows, D = 5120):
rmsnorm_rope on q / k as column slices of the fused q|k|v buffer (ld = 3D) and on a contiguous
cross-attention q.  Run once per library (VSTYLER_LIB selects it); writes a sha256 of the outputs to gpurun_out/rownorm_<tag>.sha so a second run can check bit-identity
against the first.

usage: python tests/probes/rownorm_ab.py <tag> [<tag-to-compare-with>]
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd")]

import torch  # noqa: E402

from vstyler import kernels as K  # noqa: E402
from vstyler.models import rope_table  # noqa: E402


def main():
    tag = sys.argv[1]
    M, D, S = 59280, 5120, 29640
    grid = (19, 30, 52)
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv0 = torch.randn(M, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(D, device="cuda", generator=g)).to(torch.bfloat16)
    rope = rope_table(device="cuda")
    qkv = qkv0.clone()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        K.rmsnorm_rope(qkv[:, :D], w, 1e-6, rope=rope, grid=grid, rows_per_batch=S)
        K.rmsnorm_rope(qkv[:, D:2 * D], w, 1e-6, rope=rope, grid=grid, rows_per_batch=S)

    run()
    out = qkv.clone()
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        st.record()
        for _ in range(20):
            run()
        en.record()
        en.synchronize()
        times.append(st.elapsed_time(en) / 40)
    t = min(times)
    gb = 2 * M * D * 2 / 1e9
    print(f"[{tag}] rmsnorm_rope fused-qkv slice: {t * 1e3:.1f} us/launch = {gb / t:.2f} TB/s")
    xc = qkv0[:, :D].contiguous()
    st.record()
    for _ in range(20):
        K.rmsnorm_rope(xc, w, 1e-6)
    en.record()
    en.synchronize()
    t = st.elapsed_time(en) / 20
    print(f"[{tag}] rmsnorm (no rope) contiguous: {t * 1e3:.1f} us/launch = {gb / t:.2f} TB/s")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    digest = hashlib.sha256(out[:, :2 * D].cpu().view(torch.int16).numpy().tobytes()).hexdigest()
    with open(os.path.join(ROOT, "gpurun_out", f"rownorm_{tag}.sha"), "w") as f:
        f.write(digest)
    if len(sys.argv) > 2:
        with open(os.path.join(ROOT, "gpurun_out", f"rownorm_{sys.argv[2]}.sha")) as f:
            same = f.read() == digest
        print(f"[{tag}] bit-identical to [{sys.argv[2]}]: {same}")
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()

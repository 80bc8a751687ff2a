"""Test-only Ulysses variants: torch re-statements of the permute kernel (CPU) and host-staged
gloo collectives (several ranks sharing one GPU).  Never used by the product path."""
import torch
import torch.distributed as dist

from vstyler.usp import CfgParallel, UlyssesGroup, _Done


def permute_ref(src, dst, batch, s_local, world, cpr, ld_local, jstride, mode, packed_ld=None):
    """Pure-torch statement of vs_ulysses_permute_rows (include/vstyler.h)."""
    B, Sl, P = batch, s_local, world

    def flat(t):      # element view of t's storage from its first element (row-strided views too)
        if t.is_contiguous():
            return t.reshape(-1)
        span = (t.shape[0] - 1) * t.stride(0) + t.shape[1] if t.dim() == 2 else t.numel()
        return t.as_strided((span,), (1,))
    src1, dst1 = flat(src), flat(dst)
    j = torch.arange(P).view(P, 1, 1, 1)
    b = torch.arange(B).view(1, B, 1, 1)
    t = torch.arange(Sl).view(1, 1, Sl, 1)
    c = torch.arange(cpr).view(1, 1, 1, cpr)
    packed = j * jstride + (b * Sl + t) * (cpr if packed_ld is None else packed_ld) + c
    local = (b * Sl + t) * ld_local + j * cpr + c
    full = (b * P * Sl + j * Sl + t) * cpr + c
    so, d = {0: (local, packed), 1: (packed, local), 2: (packed, full), 3: (full, packed)}[mode]
    dst1[d.reshape(-1)] = src1[so.reshape(-1)]
    return dst


class CpuUlysses(UlyssesGroup):
    """Ulysses exchange on CPU tensors with gloo; attention by a supplied function."""
    capturable = False

    def __init__(self, attn_fn, group=None):
        super().__init__(group)
        self.attn_fn = attn_fn

    def _permute(self, src, dst, batch, s_local, cpr, ld_local, jstride, mode, packed_ld=None):
        permute_ref(src, dst, batch, s_local, self.world_size, cpr, ld_local, jstride, mode, packed_ld)

    def _attention(self, q, k, v, o, heads, batch):
        o.copy_(self.attn_fn(q, k, v, heads, batch))

    def _all_gather(self, recv, send):
        self.collective_calls += 1
        parts = list(recv.chunk(self.world_size))
        dist.all_gather(parts, send.contiguous(), group=self.group)


class HostStagedUlysses(UlyssesGroup):
    """The product UlyssesGroup (HIP permutes + HIP attention) with its collectives staged through
    host memory over gloo, so several ranks can share one GPU in a test (host syncs: not capturable
    into a hipGraph)."""
    capturable = False

    def _all_to_all(self, recv, send):
        self.collective_calls += 1
        torch.cuda.synchronize()
        r = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(r, send.cpu(), group=self.group)
        recv.copy_(r)
        return _Done()

    def _all_gather(self, recv, send):
        self.collective_calls += 1
        torch.cuda.synchronize()
        parts = [torch.empty(send.shape, dtype=send.dtype) for _ in range(self.world_size)]
        dist.all_gather(parts, send.cpu().contiguous(), group=self.group)
        recv.copy_(torch.cat(parts))


class HostStagedCfgParallel(CfgParallel):
    """The product CfgParallel with host-staged gloo collectives (Ulysses halves: HostStagedUlysses),
    so its ranks can share one GPU in a test."""
    capturable = False

    def __init__(self, group=None):
        super().__init__(group, ulysses_cls=HostStagedUlysses)

    def gather_cfg(self, out_pair, out_local):
        torch.cuda.synchronize()
        self.collective_calls += 1
        parts = [torch.empty(out_local.shape, dtype=out_local.dtype) for _ in range(2)]
        dist.all_gather(parts, out_local.cpu().contiguous(), group=self.pair_group)
        out_pair.copy_(torch.cat(parts))

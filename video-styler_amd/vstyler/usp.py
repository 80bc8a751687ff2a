"""Ulysses sequence parallelism over RCCL (torch.distributed 'nccl' == RCCL on ROCm).

Reference: initialize_usp / enable_usp (diffsynth/pipelines/wan_video_new.py:313-338), token
chunking (:1412-1417, :1447-1449), head all_gather (:1459-1462), usp_attn_forward
(diffsynth/distributed/xdit_context_parallel.py:110-131, xfuser/yunchang Ulysses all-to-all).

MI355X design: one process per GPU; the token axis is sharded contiguously (rank r owns tokens
[r*S/p, (r+1)*S/p) of every batch element) for the main AND the VACE blocks (the reference leaves
VACE unsharded); per self-attention ONE all_to_all_single carries q|k|v packed together and one
carries the output back; layout transforms are the vs_ulysses_permute kernel.  Requires
S % p == 0 and heads % p == 0 (asserted instead of the reference's silent zero padding).
"""
import os

import torch
import torch.distributed as dist

from . import kernels as K
from .models import RunCtx

_DEFAULT = None


def init_distributed():
    """wan_video_new.py:313-323: env:// rendezvous, one process per GPU; returns the local rank."""
    if not dist.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend, init_method="env://")
    local_rank = int(os.environ.get("LOCAL_RANK", dist.get_rank()))
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    return local_rank


def get_default_group():
    global _DEFAULT
    if _DEFAULT is None and dist.is_initialized():
        _DEFAULT = UlyssesGroup()
    return _DEFAULT


class UlyssesGroup:
    def __init__(self, group=None):
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    # -------------------------------------------------------------- layout helpers (kernels)
    def _permute(self, src, dst, batch, s_local, cpr, ld_local, jstride, mode):
        K.ulysses_permute(src, dst, batch, s_local, self.world_size, cpr, ld_local, jstride, mode)

    def _attention(self, q, k, v, o, heads, batch):
        from .models import TIMER
        ev = TIMER.start("self_attn")
        K.attention(q, k, v, o, heads, batch)
        TIMER.stop(ev)

    def _all_to_all(self, recv, send):
        dist.all_to_all_single(recv, send, group=self.group)

    def _all_gather(self, recv, send):
        dist.all_gather_into_tensor(recv, send, group=self.group)

    # -------------------------------------------------------------- token sharding
    def shard_tokens(self, x, vace_x, rc):
        P, B, S = self.world_size, rc.batch, rc.seq
        if S % P:
            raise ValueError(f"Ulysses SP needs tokens % world == 0 (S={S}, world={P})")
        Sl = S // P
        D = x.shape[1]
        ws = rc.ws

        def take(t, name):
            out = ws.get(name, (B * Sl, D))
            src = t.view(B, S, D)[:, self.rank * Sl:(self.rank + 1) * Sl]
            out.view(B, Sl, D).copy_(src)
            return out

        xl = take(x, "sp_x")
        vl = take(vace_x, "sp_vace") if vace_x is not None else None
        rc2 = RunCtx(B, Sl, rc.grid, rc.rope, rc.ctx, rc.ctx_len, ws, sp=self, token_offset=self.rank * Sl)
        rc2.full_seq = S
        return xl, vl, rc2

    def gather_tokens(self, out, rc):
        """[B*Sl, C] per rank -> [B*S, C] on every rank (the head all_gather)."""
        P, B, Sl = self.world_size, rc.batch, rc.seq
        C = out.shape[1]
        ws = rc.ws
        packed = ws.get("sp_gather", (P * B * Sl, C))
        self._all_gather(packed, out.contiguous())
        full = ws.get("sp_gather_full", (B * P * Sl, C))
        self._permute(packed, full, B, Sl, C, C, B * Sl * C, 2)
        return full

    # -------------------------------------------------------------- attention
    def attention(self, q, k, v, o, num_heads, batch):
        """Local q/k/v/o [B*Sl, H*128] -> all-to-all -> attention over all S tokens for H/p heads ->
        all-to-all back into o."""
        P = self.world_size
        if num_heads % P:
            raise ValueError(f"Ulysses SP needs heads % world == 0 (heads={num_heads}, world={P})")
        M, D = q.shape
        B = batch
        Sl = M // B
        Hp = num_heads // P
        cpr = Hp * 128
        ws_ = _ws_of(q)
        chunk = B * Sl * cpr                     # elements of one tensor per rank chunk
        send = ws_.get("sp_send", (P * 3 * chunk,))
        recv = ws_.get("sp_recv", (P * 3 * chunk,))
        for i, t in enumerate((q, k, v)):
            self._permute(t, send[i * chunk:], B, Sl, cpr, D, 3 * chunk, 0)
        self._all_to_all(recv, send)
        full = ws_.get("sp_full", (3, B * P * Sl, cpr))
        for i in range(3):
            self._permute(recv[i * chunk:], full[i], B, Sl, cpr, D, 3 * chunk, 2)
        of = ws_.get("sp_out_full", (B * P * Sl, cpr))
        self._attention(full[0], full[1], full[2], of, Hp, B)
        send2 = ws_.get("sp_send2", (P * chunk,))
        recv2 = ws_.get("sp_recv2", (P * chunk,))
        self._permute(of, send2, B, Sl, cpr, D, chunk, 3)
        self._all_to_all(recv2, send2)
        self._permute(recv2, o, B, Sl, cpr, D, chunk, 1)
        return o


_WS_BY_DEV = {}


def _ws_of(t):
    from .models import Workspace
    key = str(t.device)
    if key not in _WS_BY_DEV:
        _WS_BY_DEV[key] = Workspace(t.device)
    return _WS_BY_DEV[key]

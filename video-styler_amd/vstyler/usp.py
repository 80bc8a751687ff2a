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
import ctypes
import os

import torch
import torch.distributed as dist

from . import kernels as K
from .models import RunCtx
from .options import host_option

_DEFAULT = None


def init_distributed():
    """wan_video_new.py:313-323: env:// rendezvous, one process per GPU; returns the local rank.
    The device is bound BEFORE the process group exists and handed to it as device_id, so RCCL's
    communicator is created on this rank's GPU (not on the guess cuda:rank % count) at the first
    collective -- barriers included."""
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    if not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend="nccl", init_method="env://",
                                    device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend="gloo", init_method="env://")
    elif torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    return local_rank


def get_default_group():
    """The parallel plan of the whole world: one UlyssesGroup over all ranks (the reference's USP,
    "0", the default), or CfgParallel when host option cfg_parallel selects it ("1": at every even
    world size, Ulysses inside each half; "auto": at world size 2 only, where Ulysses would send half of
    every q|k|v over one xGMI link per block while CFG parallelism needs one 2-sample velocity
    exchange per step).  CfgParallel stays opt-in until a multi-GPU RCCL run has shown its output
    equal to the single-GPU forward (the tests cover it with host-staged collectives)."""
    global _DEFAULT
    if _DEFAULT is None and dist.is_initialized():
        mode = host_option("cfg_parallel")
        world = dist.get_world_size()
        if world % 2 == 0 and (mode == "1" or (mode == "auto" and world == 2)):
            _DEFAULT = CfgParallel()
        else:
            _DEFAULT = UlyssesGroup()
    return _DEFAULT


class _Done:
    def wait(self):
        pass


class _EventWork:
    """Handle of an exchange enqueued on the native comm stream: wait() makes the current stream
    wait for it (no host sync), as torch's async NCCL work does."""
    __slots__ = ("ev",)

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class NativeComm:
    """RCCL through libvstyler's own C ABI (vs_sp_* in include/vstyler.h) instead of
    torch.distributed's process group -- the path a non-Python host binds.  torch.distributed is
    used once, to hand rank 0's RCCL unique id to the other ranks.  Every collective of the
    communicator runs on ONE dedicated stream, ordered after the work enqueued so far on the caller's
    stream (RCCL's async pattern), so collectives of one communicator never reorder; all_gather then
    makes the caller's stream wait for it (synchronous to the caller, as torch's all_gather).  The
    communicator is destroyed by close() or when the object is collected.  Selected with host
    option sp_comm=native."""

    def __init__(self, group=None, stream=None):
        from . import _lib
        self._lib = _lib
        lib = _lib.load()
        self.handle = ctypes.c_void_p()
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            self._check(lib.vs_sp_unique_id(uid))
        box = [uid.raw if self.rank == 0 else None]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(box, src=src, group=group)
        uid = ctypes.create_string_buffer(box[0], 128)
        self._check(lib.vs_sp_init(self.rank, self.world, uid, torch.cuda.current_device(),
                                   ctypes.byref(self.handle)))
        # stream="side" (default): the collectives run on a stream of their own, ordered after the
        # caller's work by events, so they overlap the compute enqueued meanwhile.  "caller"
        # (host option sp_comm_stream=caller): on the caller's stream, in order with the compute.
        # hipGraph capture: RCCL on a side stream FORKED into a capture segfaults in
        # hipStreamEndCapture on this image's HIP 7.0 (torch's ProcessGroupNCCL stream and this
        # class's own alike; profiles/r3/sp_graph_probe_faulthandler.log), while RCCL on the capture's
        # ORIGIN stream captures and replays bit-identical (sp_graph_probe_caller_stream.log).  So the
        # denoising step's capture inverts the fork instead (pipeline.DenoiseStepper): the comm stream
        # is bound to the capture origin (bind_stream) and the compute runs on a stream forked from
        # it -- the same event-ordered overlap, with RCCL where the capture accepts it.
        if stream is None:
            stream = host_option("sp_comm_stream")
        if stream not in ("caller", "side"):
            raise ValueError(f"sp_comm_stream must be 'caller' or 'side', not {stream!r}")
        self.stream = None if stream == "caller" else torch.cuda.Stream()

    @property
    def capturable(self):
        """On the caller's stream, or on a side stream the step's capture binds to its origin --
        DenoiseStepper.capture refuses to capture while an open side-stream communicator reachable
        from the step's plan is not bound to the capture stream (unbound_side_comms), whatever plan
        attribute holds it."""
        return True

    @property
    def is_open(self):
        return bool(getattr(self, "handle", None))

    def bind_stream(self, stream):
        """Run the side-stream collectives on `stream` (the capture origin of DenoiseStepper);
        returns the previous stream.  No effect in caller mode."""
        old = self.stream
        if old is not None:
            self.stream = stream
        return old

    def _check(self, code):
        if code != 0:
            lib = self._lib.load()
            raise RuntimeError(f"vstyler SP comm error {code}: {lib.vs_strerror(code).decode()} "
                               f"({lib.vs_sp_last_error().decode()})")

    def _bytes_per_rank(self, t):
        nbytes = t.numel() * t.element_size()
        if nbytes % self.world:
            raise ValueError(f"exchange of {nbytes} bytes does not split over {self.world} ranks")
        return nbytes // self.world

    def all_to_all(self, recv, send):
        if self.stream is None:
            self._check(self._lib.load().vs_sp_all_to_all(self.handle, send.data_ptr(), recv.data_ptr(),
                                                          self._bytes_per_rank(send),
                                                          torch.cuda.current_stream().cuda_stream))
            return _Done()
        self.stream.wait_stream(torch.cuda.current_stream())
        self._check(self._lib.load().vs_sp_all_to_all(self.handle, send.data_ptr(), recv.data_ptr(),
                                                      self._bytes_per_rank(send), self.stream.cuda_stream))
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _EventWork(ev)

    def all_gather(self, recv, send):
        cur = torch.cuda.current_stream()
        if self.stream is None:
            self._check(self._lib.load().vs_sp_all_gather(self.handle, send.data_ptr(), recv.data_ptr(),
                                                          send.numel() * send.element_size(), cur.cuda_stream))
            return
        self.stream.wait_stream(cur)
        self._check(self._lib.load().vs_sp_all_gather(self.handle, send.data_ptr(), recv.data_ptr(),
                                                      send.numel() * send.element_size(),
                                                      self.stream.cuda_stream))
        cur.wait_stream(self.stream)

    def close(self):
        if getattr(self, "handle", None):
            self._check(self._lib.load().vs_sp_comm_destroy(self.handle))
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:       # interpreter shutdown: the library may already be unloaded
            pass


class _Exchange:
    """In-flight state of one Ulysses attention (one micro-batch of one block)."""
    __slots__ = ("q", "B", "Sl", "Hp", "cpr", "D", "chunk", "tag", "ws", "work", "work2", "recv2", "rows")


class UlyssesGroup:
    """overlap: split the CFG batch into per-sample micro-batches inside each block so one half's
    all-to-alls (async on RCCL's stream) run under the other half's GEMMs / attention / FFN
    (host option sp_overlap=0 disables).  force_collectives: run the sharded path (permutes and RCCL
    collectives) even at world size 1, where model_fn_wan_video otherwise takes the plain path
    (tests use it to drive the real collectives on a one-GPU box).  comm: "torch" (torch.distributed
    on the process group, default) or "native" (NativeComm: RCCL through libvstyler's vs_sp_* ABI);
    default from host option sp_comm."""

    @property
    def capturable(self):
        """The step's hipGraph may capture this plan's collectives: RCCL through vs_sp_* on the
        caller's stream (NativeComm.capturable); torch.distributed's RCCL runs on the process
        group's own stream, which the capture does not survive (NativeComm's comment)."""
        return self.native is not None and self.native.capturable

    def __init__(self, group=None, force_collectives=False, comm=None):
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.overlap = bool(host_option("sp_overlap"))
        self.force_collectives = force_collectives
        self.collective_calls = 0
        comm = comm or host_option("sp_comm")
        if comm not in ("torch", "native"):
            raise ValueError(f"sp_comm must be 'torch' or 'native', not {comm!r}")
        self.native = NativeComm(group) if comm == "native" else None

    # -------------------------------------------------------------- layout helpers (kernels)
    def _permute(self, src, dst, batch, s_local, cpr, ld_local, jstride, mode, packed_ld=None):
        K.ulysses_permute(src, dst, batch, s_local, self.world_size, cpr, ld_local, jstride, mode, packed_ld)

    def _attention(self, q, k, v, o, heads, batch):
        from .models import TIMER, attn_flops
        ev = TIMER.start("self_attn", attn_flops(q, k, batch))
        K.attention(q, k, v, o, heads, batch)
        TIMER.stop(ev)

    def _all_to_all(self, recv, send):
        """Asynchronous: RCCL's stream waits for the work enqueued so far on the current stream;
        the returned handle's wait() makes the current stream wait for the exchange."""
        self.collective_calls += 1
        if self.native is not None:
            return self.native.all_to_all(recv, send)
        return dist.all_to_all_single(recv, send, group=self.group, async_op=True)

    def _all_gather(self, recv, send):
        self.collective_calls += 1
        if self.native is not None:
            self.native.all_gather(recv, send)
            return
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

    # -------------------------------------------------------------- attention (3 stages)
    def exchange_start(self, q, k, v, num_heads, batch, tag=""):
        """Pack local q|k|v [B*Sl, H*128] per destination rank and start the all-to-all."""
        P = self.world_size
        if num_heads % P:
            raise ValueError(f"Ulysses SP needs heads % world == 0 (heads={num_heads}, world={P})")
        e = _Exchange()
        M, D = q.shape
        e.q, e.B, e.D, e.tag = q, batch, D, tag
        e.Sl = M // batch
        e.Hp = num_heads // P
        e.cpr = e.Hp * 128
        e.ws = _ws_of(q)
        e.chunk = batch * e.Sl * e.cpr                # elements of one tensor per rank chunk
        send = e.ws.get("sp_send" + tag, (P * 3 * e.chunk,))
        recv = e.ws.get("sp_recv" + tag, (P * 3 * e.chunk,))
        # one sample: chunk j holds its tokens' q|k|v rows for rank j's heads ([Sl, 3 cpr]), so the
        # received buffer is the whole sequence's q|k|v rows in token order -- attention reads it in
        # place.  Several samples: chunk j is [q | k | v] of [B, Sl, cpr] each, re-laid out on arrival.
        e.rows = batch == 1 and bool(host_option("sp_rows"))
        for i, t in enumerate((q, k, v)):     # row stride: q/k/v may be column slices of a fused q|k|v
            if e.rows:
                self._permute(t, send[i * e.cpr:], 1, e.Sl, e.cpr, t.stride(0), 3 * e.chunk, 0, 3 * e.cpr)
            else:
                self._permute(t, send[i * e.chunk:], batch, e.Sl, e.cpr, t.stride(0), 3 * e.chunk, 0)
        e.work = self._all_to_all(recv, send)
        return e

    def attend(self, e):
        """Wait for q|k|v, attention over all S tokens for H/p heads, start the return exchange."""
        P, B, Sl, cpr, D, chunk, ws = self.world_size, e.B, e.Sl, e.cpr, e.D, e.chunk, e.ws
        e.work.wait()
        recv = ws.get("sp_recv" + e.tag, (P * 3 * chunk,))
        of = ws.get("sp_out_full" + e.tag, (B * P * Sl, cpr))
        e.recv2 = ws.get("sp_recv2" + e.tag, (P * chunk,))
        if e.rows:
            # [P Sl, 3 cpr] in token order; O [P Sl, cpr] is already the return exchange's packing
            rows = recv.view(P * Sl, 3 * cpr)
            self._attention(rows[:, :cpr], rows[:, cpr:2 * cpr], rows[:, 2 * cpr:], of, e.Hp, 1)
            e.work2 = self._all_to_all(e.recv2, of.view(-1))
            return e
        full = ws.get("sp_full" + e.tag, (3, B * P * Sl, cpr))
        for i in range(3):
            self._permute(recv[i * chunk:], full[i], B, Sl, cpr, D, 3 * chunk, 2)
        self._attention(full[0], full[1], full[2], of, e.Hp, B)
        send2 = ws.get("sp_send2" + e.tag, (P * chunk,))
        self._permute(of, send2, B, Sl, cpr, D, chunk, 3)
        e.work2 = self._all_to_all(e.recv2, send2)
        return e

    def finish(self, e, o):
        """Wait for the head-sharded output and scatter it back into local rows o [B*Sl, H*128]."""
        e.work2.wait()
        self._permute(e.recv2, o, e.B, e.Sl, e.cpr, e.D, e.chunk, 1)
        return o

    def attention(self, q, k, v, o, num_heads, batch):
        """Local q/k/v/o [B*Sl, H*128] -> all-to-all -> attention over all S tokens for H/p heads ->
        all-to-all back into o (the three stages back to back)."""
        return self.finish(self.attend(self.exchange_start(q, k, v, num_heads, batch)), o)


_WS_BY_DEV = {}


def reachable_native_comms(plan, depth=4):
    """Every open NativeComm reachable from a parallel plan through its attributes (any name, lists,
    tuples and dicts included, `depth` levels deep)."""
    out, seen = [], set()

    def visit(o, d):
        if o is None or id(o) in seen or d < 0 or isinstance(o, (str, bytes, int, float, torch.Tensor)):
            return
        seen.add(id(o))
        if isinstance(o, NativeComm):
            if o.is_open:
                out.append(o)
            return
        if isinstance(o, dict):
            items = list(o.values())
        elif isinstance(o, (list, tuple, set)):
            items = list(o)
        elif hasattr(o, "__dict__"):
            items = list(vars(o).values())
        else:
            return
        for x in items:
            visit(x, d - 1)
    visit(plan, depth)
    return out


def unbound_side_comms(stream, plan):
    """The open side-stream NativeComm objects of `plan` (reachable_native_comms) whose collectives
    would NOT run on `stream` (a graph capture's origin): RCCL forked into a capture from any other
    stream segfaulted in hipStreamEndCapture (NativeComm's comment), so a capture must see this list
    empty.  Communicators of other plans are not launched by the step and do not count."""
    return [c for c in reachable_native_comms(plan) if c.stream is not None and c.stream != stream]


def plan_native_comms(plan):
    """Every NativeComm of a parallel plan (Ulysses groups, CfgParallel's pair exchange and its
    sub-plans) whose collectives run on a side stream: the ones a step capture must bind."""
    out, seen = [], set()

    def visit(p):
        if p is None or id(p) in seen:
            return
        seen.add(id(p))
        for name in ("native", "pair_native"):
            c = getattr(p, name, None)
            if c is not None and c.stream is not None and c not in out:
                out.append(c)
        for name in ("ulysses", "full"):
            visit(getattr(p, name, None))
    visit(plan)
    return out


def _ws_of(t):
    from .models import Workspace
    key = str(t.device)
    if key not in _WS_BY_DEV:
        _WS_BY_DEV[key] = Workspace(t.device)
    return _WS_BY_DEV[key]


class CfgParallel:
    """CFG parallelism x Ulysses (SURVEY.md §8e's optional extra; not in the reference, whose USP is
    Ulysses only).  World W = 2u: ranks [c*u, (c+1)*u) of `group` compute CFG sample c (c = 0 the
    positive prompt, 1 the negative) as a batch-1 forward, its token axis sharded by Ulysses over
    those u ranks (u = 1: no exchange inside the forward at all); after the head, rank j of half 0
    and rank j of half 1 all-gather their samples' velocities, so every rank returns the batch-2
    output of the single-GPU forward (model_fn_wan_video does this when handed a CfgParallel).
    Per-row work is that of the batch-2 forward.  Batch-1 forwards (no CFG, cfg_scale 1) and
    TeaCache steps fall back to `self.full`, a Ulysses group over all W ranks.  comm as UlyssesGroup."""

    def __init__(self, group=None, comm=None, ulysses_cls=None):
        ulysses_cls = ulysses_cls or UlyssesGroup
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world_size % 2:
            raise ValueError(f"CFG parallelism needs an even world size, not {self.world_size}")
        u = self.world_size // 2
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world_size))
        self.cfg_rank, self.half_rank = divmod(self.rank, u)
        # every rank creates every subgroup, in the same order (torch.distributed.new_group contract)
        halves = [dist.new_group([ranks[c * u + j] for j in range(u)]) for c in range(2)] if u > 1 else None
        pairs = [dist.new_group([ranks[j], ranks[u + j]]) for j in range(u)]
        self.pair_group = pairs[self.half_rank]
        self.ulysses = ulysses_cls(halves[self.cfg_rank], comm=comm) if u > 1 else None
        self.full = ulysses_cls(group, comm=comm)
        comm = comm or host_option("sp_comm")
        # the velocity exchange goes through the same comm kind as the Ulysses exchanges
        self.pair_native = NativeComm(self.pair_group) if comm == "native" else None
        self.collective_calls = 0

    @property
    def capturable(self):
        """The velocity exchange is capturable as UlyssesGroup's (its sub-plans are checked apart)."""
        return self.pair_native is not None and self.pair_native.capturable

    def gather_cfg(self, out_pair, out_local):
        """out_local [1, ...] of this rank's CFG sample -> out_pair [2, ...] (sample 0, sample 1)."""
        self.collective_calls += 1
        if self.pair_native is not None:
            self.pair_native.all_gather(out_pair, out_local.contiguous())
            return
        dist.all_gather_into_tensor(out_pair, out_local.contiguous(), group=self.pair_group)

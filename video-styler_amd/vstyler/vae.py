"""Wan2.1 causal 3-D VAE on gfx950 (replaces diffsynth/models/wan_video_vae.py, Wan2.1 part).

Drop-in surface: `WanVideoVAE.encode(videos, device, tiled, tile_size, tile_stride)` and
`.decode(hidden_states, device, tiled, tile_size, tile_stride)` (wan_video_vae.py:1218-1247), same
tiling rule, same blend arithmetic, same latent normalisation; parameters load by the reference's
state-dict names (registry md5 `ccc42284…`, configs/model_config.py:164).

Execution is MI355X-first, not a translation of the reference's chunk loop:
* Whole-sequence form.  The reference encodes chunks of [1, 4, 4, ...] frames (decodes one latent
  frame at a time) and threads a 2-frame feature cache through every causal conv
  (:44-52,283-301,984-1034).  That cache makes each causal conv equal to one conv over the whole
  sequence with 2 leading zero frames; the two exceptions are reproduced exactly: downsample3d
  passes frame 0 through and convolves frames (2j-2, 2j-1, 2j) for j >= 1 (:162-173), upsample3d
  passes frame 0 through and runs its time conv over frames 1.. only, causally zero padded
  (the 'Rep' sentinel, :122-156).  Each layer is then one launch over all frames of all tiles.
* All tiles of one shape are batched into one activation tensor (n = tiles), so a launch has
  thousands of workgroups even at the 1/8-resolution levels.
* Channels-last (NTHWC) bf16 activations; every conv is `vs_vae_conv` (implicit-GEMM MFMA with
  padding/upsample fused into the gather), RMS_norm+SiLU is one pass (`vs_vae_rmsnorm`), the
  1x1 convs of VideoVAE_ are the same kernel.  Tiles never leave HBM (the reference moves each
  tile host<->device, :1125-1126,1177-1178); blending follows the reference's bf16 task order.
"""
import math

import torch

from . import _lib
from ._lib import VsConv3d

BF16 = torch.bfloat16

# wan_video_vae.py:1063-1070
VAE_MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
            0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
VAE_STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
           3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]


def _r32(c):
    return (c + 31) // 32 * 32


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class ConvW:
    """A conv weight re-laid out once at load for the implicit GEMM: [cout][kt][kh][kw][cin_pad]
    (input channels padded with zeros to a multiple of 32)."""

    def __init__(self, weight, bias, device):
        w = weight.detach()
        if w.dim() == 4:  # nn.Conv2d
            w = w.unsqueeze(2)
        co, ci, kt, kh, kw = w.shape
        self.cout, self.cin, self.k, self.cin_real = co, _r32(ci), (kt, kh, kw), ci
        wp = torch.zeros((co, kt, kh, kw, self.cin), dtype=BF16, device=device)
        wp[..., :ci] = w.to(device=device, dtype=BF16).permute(0, 2, 3, 4, 1)
        self.w = wp.reshape(co, -1).contiguous()
        self.bias = None if bias is None else bias.detach().to(device=device, dtype=BF16).contiguous()


# algorithmic FLOPs issued through conv()/batched_gemm() (real channel counts, no padding);
# bench/probe code reads and resets it.
FLOPS = [0]


def conv(x, cw, out_thw, *, stride=(1, 1, 1), pad=(0, 0, 0), up2=False, t_lo=0, y=None, t_mul=1,
         t_add=0, split=0, res=None):
    """One vs_vae_conv launch.  x: [n, t, h, w, c] channels-last bf16 (c >= cw.cin, padded channels
    zero); returns y [n, T_y, h_out, w_out, cout] (allocated unless given)."""
    n, t, h, w, c = x.shape
    if c != cw.cin:
        raise ValueError(f"conv: input has {c} channels, weight expects {cw.cin}")
    if not x.is_contiguous():
        raise ValueError("conv: input must be contiguous NTHWC")
    t_out, h_out, w_out = out_thw
    if y is None:
        y = torch.empty((n, t_out, h_out, w_out, cw.cout), dtype=BF16, device=x.device)
    p = VsConv3d()
    p.x, p.x_zs, p.x_ns, p.ldx = x.data_ptr(), 0, x.stride(0), c
    p.n, p.t_in, p.h_in, p.w_in, p.cin = n, t, h, w, c
    p.kt, p.kh, p.kw = cw.k
    p.st, p.sh, p.sw = stride
    p.pt, p.ph, p.pw = pad
    p.up2, p.t_lo = int(up2), t_lo
    p.t_out, p.h_out, p.w_out = t_out, h_out, w_out
    p.w, p.w_zs, p.ldw = cw.w.data_ptr(), 0, cw.w.shape[1]
    p.bias = None if cw.bias is None else cw.bias.data_ptr()
    p.cout = cw.cout
    p.y, p.y_zs, p.y_ns, p.ldy = y.data_ptr(), 0, y.stride(0), y.shape[-1]
    p.t_mul, p.t_add, p.split, p.out_f32, p.alpha = t_mul, t_add, split, 0, 1.0
    if res is not None:
        if res.shape != y.shape or not res.is_contiguous():
            raise ValueError("conv: residual must match the output geometry")
        p.res = res.data_ptr()
    p.nz = 1
    _lib.check(_lib.load().vs_vae_conv(p, _stream(x)))
    FLOPS[0] += 2 * n * t_out * h_out * w_out * cw.cout * cw.cin_real * cw.k[0] * cw.k[1] * cw.k[2]
    return y


def batched_gemm(a, a_zs, lda, rows, k, b, b_zs, ldb, n_out, y, y_zs, ldy, nz, out_f32=False, alpha=1.0):
    """C[z][r][j] = alpha * sum_k A[z][r][k] B[z][j][k] through the conv kernel's GEMM mode."""
    p = VsConv3d()
    p.x, p.x_zs, p.x_ns, p.ldx = a.data_ptr(), a_zs, 0, lda
    p.n, p.t_in, p.h_in, p.w_in, p.cin = 1, 1, 1, rows, k
    p.kt = p.kh = p.kw = p.st = p.sh = p.sw = 1
    p.pt = p.ph = p.pw = p.up2 = p.t_lo = 0
    p.t_out, p.h_out, p.w_out = 1, 1, rows
    p.w, p.w_zs, p.ldw = b.data_ptr(), b_zs, ldb
    p.bias, p.cout = None, n_out
    p.y, p.y_zs, p.y_ns, p.ldy = y.data_ptr(), y_zs, 0, ldy
    p.t_mul, p.t_add, p.split, p.out_f32, p.alpha = 1, 0, 0, int(out_f32), alpha
    p.res, p.nz = None, nz
    _lib.check(_lib.load().vs_vae_conv(p, _stream(a)))
    FLOPS[0] += 2 * nz * rows * n_out * k


def rmsnorm(x, gamma, silu, out=None):
    """RMS_norm (+SiLU) over the channel dim of a channels-last tensor (in place if out is x)."""
    c = x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    _lib.check(_lib.load().vs_vae_rmsnorm(x.data_ptr(), c, out.data_ptr(), c, gamma.data_ptr(),
                                          x.numel() // c, c, int(silu), _stream(x)))
    return out


def copy_first_frame(src, dst):
    n, t, h, w, c = src.shape
    _lib.check(_lib.load().vs_vae_copy_frames(src.data_ptr(), src.stride(0), dst.data_ptr(), dst.stride(0),
                                              n, h * w * c, _stream(src)))


class WanVideoVAE:
    """Replaces WanVideoVAE (wan_video_vae.py:1058-1252) for the Wan2.1 16-channel VAE."""

    upsampling_factor = 8

    def __init__(self, z_dim=16, dim=96, dim_mult=(1, 2, 4, 4), num_res_blocks=2,
                 temperal_downsample=(False, True, True), device="cuda", attn_bytes=2 << 30,
                 max_tile_batch=16):
        self.z_dim, self.dim, self.dim_mult, self.nrb = z_dim, dim, tuple(dim_mult), num_res_blocks
        self.temperal_downsample = tuple(temperal_downsample)
        self.device = torch.device(device)
        self.attn_bytes = attn_bytes
        self.max_tile_batch = max_tile_batch
        self.mean = torch.tensor(VAE_MEAN[:z_dim]).to(BF16).to(self.device)
        self.inv_std = (1.0 / torch.tensor(VAE_STD[:z_dim])).to(BF16).to(self.device)
        self.params = {}
        self.cw = {}
        self.enc_layers, self.enc_dims = self._encoder_layers()
        self.dec_layers, self.dec_dims = self._decoder_layers()

    # ---------------------------------------------------------------- structure (:517-567, :736-787)
    def _encoder_layers(self):
        dims = [self.dim * u for u in (1,) + self.dim_mult]
        out, k = [], 0
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            for _ in range(self.nrb):
                out.append(("res", f"model.encoder.downsamples.{k}.", (a, b)))
                k, a = k + 1, b
            if i != len(self.dim_mult) - 1:
                out.append(("resample", f"model.encoder.downsamples.{k}.",
                            (b, "downsample3d" if self.temperal_downsample[i] else "downsample2d")))
                k += 1
        return out, dims

    def _decoder_layers(self):
        dims = [self.dim * u for u in (self.dim_mult[-1],) + self.dim_mult[::-1]]
        tu = self.temperal_downsample[::-1]
        out, k = [], 0
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            if i in (1, 2, 3):
                a //= 2
            for _ in range(self.nrb + 1):
                out.append(("res", f"model.decoder.upsamples.{k}.", (a, b)))
                k, a = k + 1, b
            if i != len(self.dim_mult) - 1:
                out.append(("resample", f"model.decoder.upsamples.{k}.",
                            (b, "upsample3d" if tu[i] else "upsample2d")))
                k += 1
        return out, dims

    # ---------------------------------------------------------------- loading
    def load_state_dict(self, state_dict):
        """Accepts the civitai file layout (keys without 'model.', or wrapped in 'model_state')
        or the converted one (WanVideoVAEStateDictConverter.from_civitai, :1260-1266)."""
        if "model_state" in state_dict:
            state_dict = state_dict["model_state"]
        sd = {(k if k.startswith("model.") else "model." + k): v for k, v in state_dict.items()}
        self.params = {}
        for k, v in sd.items():
            if k.endswith("gamma"):
                self.params[k] = v.detach().reshape(-1).to(device=self.device, dtype=BF16).contiguous()
        self.cw = {}
        for k in sd:
            if k.endswith(".weight"):
                base = k[: -len("weight")]
                self.cw[base] = ConvW(sd[k], sd.get(base + "bias"), self.device)
        return self

    def state_dict_shapes(self):
        """The civitai file layout of this configuration (keys without 'model.')."""
        d, z = {}, self.z_dim

        def res(p, i, o):
            d[p + "residual.0.gamma"] = (i, 1, 1, 1)
            d[p + "residual.2.weight"], d[p + "residual.2.bias"] = (o, i, 3, 3, 3), (o,)
            d[p + "residual.3.gamma"] = (o, 1, 1, 1)
            d[p + "residual.6.weight"], d[p + "residual.6.bias"] = (o, o, 3, 3, 3), (o,)
            if i != o:
                d[p + "shortcut.weight"], d[p + "shortcut.bias"] = (o, i, 1, 1, 1), (o,)

        def attn(p, c):
            d[p + "norm.gamma"] = (c, 1, 1)
            d[p + "to_qkv.weight"], d[p + "to_qkv.bias"] = (3 * c, c, 1, 1), (3 * c,)
            d[p + "proj.weight"], d[p + "proj.bias"] = (c, c, 1, 1), (c,)

        def resample(p, c, mode):
            co = c // 2 if mode.startswith("up") else c
            d[p + "resample.1.weight"], d[p + "resample.1.bias"] = (co, c, 3, 3), (co,)
            if mode.endswith("3d"):
                ct = 2 * c if mode == "upsample3d" else c
                d[p + "time_conv.weight"], d[p + "time_conv.bias"] = (ct, c, 3, 1, 1), (ct,)

        strip = lambda p: p[len("model."):]  # noqa: E731
        e0, top = self.enc_dims[0], self.enc_dims[-1]
        d["encoder.conv1.weight"], d["encoder.conv1.bias"] = (e0, 3, 3, 3, 3), (e0,)
        for kind, p, args in self.enc_layers:
            (res if kind == "res" else resample)(strip(p), *args)
        res("encoder.middle.0.", top, top)
        attn("encoder.middle.1.", top)
        res("encoder.middle.2.", top, top)
        d["encoder.head.0.gamma"] = (top, 1, 1, 1)
        d["encoder.head.2.weight"], d["encoder.head.2.bias"] = (2 * z, top, 3, 3, 3), (2 * z,)
        d["conv1.weight"], d["conv1.bias"] = (2 * z, 2 * z, 1, 1, 1), (2 * z,)
        d["conv2.weight"], d["conv2.bias"] = (z, z, 1, 1, 1), (z,)
        d0, dl = self.dec_dims[0], self.dec_dims[-1]
        d["decoder.conv1.weight"], d["decoder.conv1.bias"] = (d0, z, 3, 3, 3), (d0,)
        res("decoder.middle.0.", d0, d0)
        attn("decoder.middle.1.", d0)
        res("decoder.middle.2.", d0, d0)
        for kind, p, args in self.dec_layers:
            (res if kind == "res" else resample)(strip(p), *args)
        d["decoder.head.0.gamma"] = (dl, 1, 1, 1)
        d["decoder.head.2.weight"], d["decoder.head.2.bias"] = (3, dl, 3, 3, 3), (3,)
        return d

    def init_random_(self, seed=6):
        """Synthetic on-device weights (bench / smoke): conv weights N(0, 1/fan_in), biases 0.01*N,
        gammas 1 + 0.1*N."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        sd = {}
        for name, shape in self.state_dict_shapes().items():
            if name.endswith("gamma"):
                t = 1.0 + 0.1 * torch.randn(shape, generator=g, device=self.device)
            elif name.endswith("bias"):
                t = 0.01 * torch.randn(shape, generator=g, device=self.device)
            else:
                fan_in = 1
                for v in shape[1:]:
                    fan_in *= v
                t = torch.randn(shape, generator=g, device=self.device) / math.sqrt(fan_in)
            sd[name] = t.to(BF16)
        return self.load_state_dict(sd)

    # ---------------------------------------------------------------- layers
    def _conv3(self, x, name, res=None):
        """CausalConv3d(k=3, padding=1) over the whole sequence (2 leading zero frames)."""
        n, t, h, w, _ = x.shape
        return conv(x, self.cw[name], (t, h, w), pad=(2, 1, 1), res=res)

    def _conv1(self, x, name, y=None):
        n, t, h, w, _ = x.shape
        return conv(x, self.cw[name], (t, h, w), y=y)

    def _res_block(self, x, p):
        """ResidualBlock (:267-301): x + conv(silu(norm(conv(silu(norm(x))))))."""
        h = self._conv1(x, p + "shortcut.") if (p + "shortcut.") in self.cw else x
        a = rmsnorm(x, self.params[p + "residual.0.gamma"], silu=True)
        a = self._conv3(a, p + "residual.2.")
        rmsnorm(a, self.params[p + "residual.3.gamma"], silu=True, out=a)
        return self._conv3(a, p + "residual.6.", res=h)

    def _attn_block(self, x, p, flash=None):
        """AttentionBlock (:304-342): per frame single-head attention over h*w tokens, d = C.  The
        flash kernel (vs_vae_attention) for C % 128 == 0 (Wan2.1: 384; flash=False selects the GEMM
        route for A/Bs), else fp32 scores + softmax + P.V through the conv kernel's GEMM mode."""
        n, t, h, w, c = x.shape
        hw, nz = h * w, n * t
        xn = rmsnorm(x, self.params[p + "norm.gamma"], silu=False)
        qkv = self._conv1(xn, p + "to_qkv.")                      # [n, t, h, w, 3c]
        del xn
        o = torch.empty((n, t, h, w, c), dtype=BF16, device=x.device)
        if flash is None:
            flash = c % 128 == 0 and c <= 384
        if flash:
            _lib.check(_lib.load().vs_vae_attention(qkv.data_ptr(), hw * 3 * c, 3 * c, o.data_ptr(), hw * c, c, nz,
                                                    hw, c, _stream(x)))
            FLOPS[0] += 4 * nz * hw * hw * c
            del qkv
            return conv(o, self.cw[p + "proj."], (t, h, w), res=x)
        hwp = _r32(hw)
        zc = max(1, min(nz, self.attn_bytes // (hw * hwp * 4)))
        s = torch.empty((zc, hw, hwp), dtype=torch.float32, device=x.device)
        pm = torch.empty((zc, hw, hwp), dtype=BF16, device=x.device)
        vt = torch.empty((zc, c, hwp), dtype=BF16, device=x.device)
        lib = _lib.load()
        st = _stream(x)
        q_all = qkv.view(nz, hw, 3 * c)
        o_all = o.view(nz, hw, c)
        for z0 in range(0, nz, zc):
            zn = min(zc, nz - z0)
            q = q_all[z0]
            batched_gemm(q, hw * 3 * c, 3 * c, hw, c, q[:, c:], hw * 3 * c, 3 * c, hw, s, hw * hwp, hwp, zn,
                         out_f32=True, alpha=1.0 / math.sqrt(c))
            _lib.check(lib.vs_vae_softmax(s.data_ptr(), hwp, pm.data_ptr(), hwp, zn * hw, hw, st))
            _lib.check(lib.vs_vae_transpose(q[:, 2 * c:].data_ptr(), hw * 3 * c, 3 * c, vt.data_ptr(), c * hwp,
                                            hwp, zn, hw, c, st))
            batched_gemm(pm, hw * hwp, hwp, hw, hwp, vt, c * hwp, hwp, c, o_all[z0], hw * c, c, zn)
        del s, pm, vt, qkv
        return conv(o, self.cw[p + "proj."], (t, h, w), res=x)

    def _resample(self, x, p, mode):
        """Resample (:82-174) in whole-sequence form."""
        n, t, h, w, c = x.shape
        if mode == "upsample3d":
            y = torch.empty((n, 1 + 2 * (t - 1), h, w, c), dtype=BF16, device=x.device)
            copy_first_frame(x, y)
            if t > 1:  # time conv over frames 1.., causal zero pad 2, channel halves -> frames 2j-1, 2j
                conv(x, self.cw[p + "time_conv."], (t - 1, h, w), pad=(1, 0, 0), t_lo=1, y=y, t_mul=2, t_add=1,
                     split=c)
            x = y
            t = x.shape[1]
        if mode.startswith("upsample"):
            return conv(x, self.cw[p + "resample.1."], (t, 2 * h, 2 * w), pad=(0, 1, 1), up2=True)
        # ZeroPad2d((0, 1, 0, 1)) + 3x3 stride 2
        ho, wo = (h + 1 - 3) // 2 + 1, (w + 1 - 3) // 2 + 1
        x = conv(x, self.cw[p + "resample.1."], (t, ho, wo), stride=(1, 2, 2))
        if mode == "downsample3d":
            to = (t - 1) // 2
            y = torch.empty((n, 1 + to, ho, wo, c), dtype=BF16, device=x.device)
            copy_first_frame(x, y)
            if to > 0:
                conv(x, self.cw[p + "time_conv."], (to, ho, wo), stride=(2, 1, 1), y=y, t_add=1)
            x = y
        return x

    def _run_layers(self, x, layers):
        for kind, p, args in layers:
            x = self._res_block(x, p) if kind == "res" else self._resample(x, p, args[1])
        return x

    def encode_tiles(self, x):
        """Encoder3d + VideoVAE_.conv1 on a batch of tiles x [n, T, H, W, 32] (RGB in channels 0-2,
        T = 1 + 4k).  Returns [n, 1 + k, H/8, W/8, 2*z_dim]; mu = channels [0, z_dim)."""
        x = self._conv3(x, "model.encoder.conv1.")
        x = self._run_layers(x, self.enc_layers)
        x = self._res_block(x, "model.encoder.middle.0.")
        x = self._attn_block(x, "model.encoder.middle.1.")
        x = self._res_block(x, "model.encoder.middle.2.")
        x = rmsnorm(x, self.params["model.encoder.head.0.gamma"], silu=True, out=x)
        x = self._conv3(x, "model.encoder.head.2.")
        return self._conv1(x, "model.conv1.")

    def decode_tiles(self, z):
        """VideoVAE_.conv2 + Decoder3d on de-normalised latent tiles z [n, T, h, w, 32] (channels
        >= z_dim zero).  Returns [n, 4T-3, 8h, 8w, 4] (RGB in channels 0-2)."""
        n, t, h, w, _ = z.shape
        x = torch.zeros((n, t, h, w, _r32(self.z_dim)), dtype=BF16, device=z.device)
        self._conv1(z, "model.conv2.", y=x)
        x = self._conv3(x, "model.decoder.conv1.")
        x = self._res_block(x, "model.decoder.middle.0.")
        x = self._attn_block(x, "model.decoder.middle.1.")
        x = self._res_block(x, "model.decoder.middle.2.")
        x = self._run_layers(x, self.dec_layers)
        x = rmsnorm(x, self.params["model.decoder.head.0.gamma"], silu=True, out=x)
        n, t, h, w, _ = x.shape
        y = torch.empty((n, t, h, w, 4), dtype=BF16, device=x.device)
        return conv(x, self.cw["model.decoder.head.2."], (t, h, w), pad=(2, 1, 1), y=y)

    # ---------------------------------------------------------------- tiling (:1081-1247)
    @staticmethod
    def tile_tasks(H, W, size, stride):
        tasks = []
        for h in range(0, H, stride[0]):
            if h - stride[0] >= 0 and h - stride[0] + size[0] >= H:
                continue
            for w in range(0, W, stride[1]):
                if w - stride[1] >= 0 and w - stride[1] + size[1] >= W:
                    continue
                tasks.append((h, h + size[0], w, w + size[1]))
        return tasks

    def _run_tasks(self, src, tasks, H, W, t_src, t_use, cpad, gather_mode, fn):
        """Gather every task's tile (batched per tile shape) and run fn on the batches.
        Returns {task index: (batch output, row)}."""
        lib = _lib.load()
        st = _stream(src)
        c = src.shape[0]
        groups = {}
        for i, (h, h_, w, w_) in enumerate(tasks):
            groups.setdefault((min(h_, H) - h, min(w_, W) - w), []).append(i)
        out = {}
        a = self.mean.data_ptr() if gather_mode else None
        b = self.inv_std.data_ptr() if gather_mode else None
        for (th, tw), idx in groups.items():
            for g0 in range(0, len(idx), self.max_tile_batch):
                ids = idx[g0:g0 + self.max_tile_batch]
                x = torch.empty((len(ids), t_use, th, tw, cpad), dtype=BF16, device=src.device)
                for j, i in enumerate(ids):
                    h, _, w, _ = tasks[i]
                    _lib.check(lib.vs_vae_tile_gather(src.data_ptr(), c, t_src, H, W, t_use, h, w, th, tw,
                                                      x[j].data_ptr(), cpad, gather_mode, a, b, st))
                y = fn(x)
                del x
                for j, i in enumerate(ids):
                    out[i] = (y, j)
        return out

    def _blend(self, tasks, outs, H, W, f_out, size, stride, c, t, ldc, clamp, mode, factor_in):
        """values/weight accumulation in task order (:1136-1152, :1188-1203), then divide."""
        lib = _lib.load()
        Ho, Wo = H * f_out if f_out >= 1 else H // factor_in, W * f_out if f_out >= 1 else W // factor_in
        any_y = outs[0][0]
        st = _stream(any_y)
        values = torch.zeros((c, t, Ho, Wo), dtype=BF16, device=any_y.device)
        weight = torch.zeros((t, Ho, Wo), dtype=BF16, device=any_y.device)
        a = self.mean.data_ptr() if mode else None
        b = self.inv_std.data_ptr() if mode else None
        for i, (h, h_, w, w_) in enumerate(tasks):
            y, j = outs[i]
            tile = y[j]
            th, tw = tile.shape[1], tile.shape[2]
            bound = (h == 0) | ((h_ >= H) << 1) | ((w == 0) << 2) | ((w_ >= W) << 3)
            if f_out >= 1:
                bw_h, bw_w = (size[0] - stride[0]) * f_out, (size[1] - stride[1]) * f_out
                h0, w0 = h * f_out, w * f_out
            else:
                bw_h, bw_w = (size[0] - stride[0]) // factor_in, (size[1] - stride[1]) // factor_in
                h0, w0 = h // factor_in, w // factor_in
            _lib.check(lib.vs_vae_tile_blend(tile.data_ptr(), ldc, c, t, th, tw, values.data_ptr(),
                                             weight.data_ptr(), Ho, Wo, h0, w0, bound, bw_h, bw_w, mode, a, b, st))
        out = torch.empty_like(values)
        _lib.check(lib.vs_vae_blend_finish(values.data_ptr(), weight.data_ptr(), out.data_ptr(), c, t * Ho * Wo,
                                           int(clamp), st))
        return out

    def _encode_one(self, video, tiled, tile_size, tile_stride):
        video = video.to(device=self.device, dtype=BF16).contiguous()  # (3, T, H, W)
        _, T, H, W = video.shape
        t_lat = 1 + (T - 1) // 4
        f = self.upsampling_factor
        if tiled:
            size = (tile_size[0] * f, tile_size[1] * f)
            stride = (tile_stride[0] * f, tile_stride[1] * f)
            tasks = self.tile_tasks(H, W, size, stride)
        else:  # single_encode == one all-bound tile (mask 1, weight 1: bit-identical)
            size, stride, tasks = (H, W), (H, W), [(0, H, 0, W)]
        outs = self._run_tasks(video, tasks, H, W, T, 1 + 4 * (t_lat - 1), 32, 0, self.encode_tiles)
        return self._blend(tasks, outs, H, W, 0, size, stride, self.z_dim, t_lat, 2 * self.z_dim, False, 1, f)

    def _decode_one(self, z, tiled, tile_size, tile_stride):
        z = z.to(device=self.device, dtype=BF16).contiguous()  # (16, T, H, W)
        _, T, H, W = z.shape
        if tiled:
            size, stride = tuple(tile_size), tuple(tile_stride)
            tasks = self.tile_tasks(H, W, size, stride)
        else:
            size, stride, tasks = (H, W), (H, W), [(0, H, 0, W)]
        outs = self._run_tasks(z, tasks, H, W, T, T, _r32(self.z_dim), 2, self.decode_tiles)
        return self._blend(tasks, outs, H, W, self.upsampling_factor, size, stride, 3, 4 * T - 3, 4, True, 0, 1)

    # ---------------------------------------------------------------- reference API (:1218-1247)
    def encode(self, videos, device=None, tiled=False, tile_size=(34, 34), tile_stride=(18, 16)):
        # the reference rebinds tile_size/tile_stride x upsampling_factor inside its loop (:1224-1225),
        # so the j-th video of a list is tiled 8^j times coarser; reproduced for drop-in results
        outs = []
        ts, st = tuple(tile_size), tuple(tile_stride)
        for v in videos:
            outs.append(self._encode_one(v, tiled, ts, st))
            if tiled:
                f = self.upsampling_factor
                ts, st = (ts[0] * f, ts[1] * f), (st[0] * f, st[1] * f)
        return torch.stack(outs)

    def decode(self, hidden_states, device=None, tiled=False, tile_size=(34, 34), tile_stride=(18, 16)):
        return torch.stack([self._decode_one(z, tiled, tile_size, tile_stride) for z in hidden_states])


def vae_output_to_u8(video):
    """BasePipeline.vae_output_to_video (utils/__init__.py:76-91) for one (3, T, H, W) bf16 video:
    returns (T, H, W, 3) uint8 on the device."""
    video = video.contiguous()
    _, T, H, W = video.shape
    out = torch.empty((T, H, W, 3), dtype=torch.uint8, device=video.device)
    _lib.check(_lib.load().vs_vae_to_u8(video.data_ptr(), out.data_ptr(), T, H, W, _stream(video)))
    return out


def frames_to_u8(frames, device):
    """A video as the reference's pipelines receive it (list of PIL images / HxWx3 uint8 arrays, or a
    (T, H, W, 3) uint8 tensor) -> contiguous (T, H, W, 3) uint8 on the device."""
    if isinstance(frames, torch.Tensor):
        t = frames
    else:
        import numpy as np
        t = torch.from_numpy(np.stack([np.asarray(f.convert("RGB") if hasattr(f, "convert") else f, dtype=np.uint8)
                                       for f in frames]))
    if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[-1] != 3:
        raise ValueError(f"expected uint8 frames (T, H, W, 3), got {tuple(t.shape)} {t.dtype}")
    return t.to(device).contiguous()


def vace_context(vae, vace_video=None, vace_video_mask=None, num_frames=None, height=None, width=None,
                 tiled=True, tile_size=(30, 52), tile_stride=(15, 26), vace_reference_image=None):
    """WanVideoUnit_VACE.process (wan_video_new.py:861-920)
    -> vace_context (1, 96, f + (T+3)//4, H/8, W/8) bf16 = [encode(inactive) | encode(reactive) | mask latents],
    preceded along time by f reference-image frames [encode(ref_j) | 0 | 0] (:896-912) when
    vace_reference_image (one image or a list of f images, each H x W) is given."""
    dev = vae.device
    v = None if vace_video is None else frames_to_u8(vace_video, dev)
    m = None if vace_video_mask is None else frames_to_u8(vace_video_mask, dev)
    ref = v if v is not None else m
    if ref is not None:
        num_frames, height, width = ref.shape[0], ref.shape[1], ref.shape[2]
    if v is not None and m is not None and v.shape != m.shape:
        raise ValueError("vace_video and vace_video_mask must have the same shape")
    T, H, W = num_frames, height, width
    inactive = torch.empty((1, 3, T, H, W), dtype=BF16, device=dev)
    reactive = torch.empty_like(inactive)
    mask0 = torch.empty((T, H, W), dtype=BF16, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    lib = _lib.load()
    _lib.check(lib.vs_vace_prepare(None if v is None else v.data_ptr(), None if m is None else m.data_ptr(),
                                   inactive.data_ptr(), reactive.data_ptr(), mask0.data_ptr(), T, H, W, st))
    t_lat = (T + 3) // 4
    nref = 0
    if vace_reference_image is not None:
        if isinstance(vace_reference_image, torch.Tensor) and vace_reference_image.dim() == 4:
            refs = vace_reference_image                     # (f, H, W, 3) uint8
        elif isinstance(vace_reference_image, (list, tuple)):
            refs = vace_reference_image
        else:
            refs = [vace_reference_image]
        r = frames_to_u8(refs, dev)
        nref = r.shape[0]
        if r.shape[1:3] != (H, W):
            raise ValueError(f"vace_reference_image must be {H}x{W}, got {tuple(r.shape[1:3])}")
        # preprocess_video of the references = the reactive output of vs_vace_prepare with mask ones
        # (v*1 + 0*0 is exact in bf16)
        r_pre = torch.empty((1, 3, nref, H, W), dtype=BF16, device=dev)
        r_tmp = torch.empty_like(r_pre)
        r_m = torch.empty((nref, H, W), dtype=BF16, device=dev)
        _lib.check(lib.vs_vace_prepare(r.data_ptr(), None, r_tmp.data_ptr(), r_pre.data_ptr(), r_m.data_ptr(),
                                       nref, H, W, st))
    out = torch.empty((1, 96, nref + t_lat, H // 8, W // 8), dtype=BF16, device=dev)
    if nref:
        rl = vae.encode([r_pre[0, :, j:j + 1] for j in range(nref)], dev, tiled=tiled, tile_size=tile_size,
                        tile_stride=tile_stride)                                      # (f, 16, 1, h, w)
        out[0, 0:16, :nref] = rl[:, :, 0].transpose(0, 1)
        out[:, 16:, :nref] = 0
    out[:, 0:16, nref:] = vae.encode(inactive, dev, tiled=tiled, tile_size=tile_size, tile_stride=tile_stride)
    out[:, 16:32, nref:] = vae.encode(reactive, dev, tiled=tiled, tile_size=tile_size, tile_stride=tile_stride)
    mlat = torch.empty((64, t_lat, H // 8, W // 8), dtype=BF16, device=dev)
    _lib.check(lib.vs_vace_mask_latents(mask0.data_ptr(), mlat.data_ptr(), T, H, W, t_lat, st))
    out[0, 32:, nref:] = mlat
    return out

"""FlowUniPCMultistepScheduler on the GPU (config 5's 4-step sampler).

Reference: denoising_enhancing/wan/utils/fm_solvers_unipc.py:22-803 (UniPC, bh2, predict-x0,
flow prediction).  The scalar coefficients are computed on the host with the reference's own fp32
0-d tensor arithmetic (sigma table, log-SNR steps, expm1, the order-2 corrector's linear solve);
every tensor update is ONE vs_unipc_update launch that reproduces the reference's fp32 op sequence
element-wise.  State (x0 predictions, last sample) stays on the device in fp32.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def _sigma_to_alpha_sigma_t(sigma):
    return 1 - sigma, sigma


def _lam(sigma):
    a, s = _sigma_to_alpha_sigma_t(sigma)
    return torch.log(a) - torch.log(s)


class FlowUniPCMultistepScheduler:
    """fm_solvers_unipc.py:79-134 (constructor) with the same defaults."""

    def __init__(self, num_train_timesteps=1000, solver_order=2, prediction_type="flow_prediction", shift=1.0,
                 use_dynamic_shifting=False, predict_x0=True, solver_type="bh2", lower_order_final=True,
                 disable_corrector=(), final_sigmas_type="zero"):
        if prediction_type != "flow_prediction" or solver_type not in ("bh1", "bh2") or not predict_x0 \
                or use_dynamic_shifting or final_sigmas_type != "zero":
            raise NotImplementedError("only the flow-prediction, predict-x0, static-shift, zero-final UniPC "
                                      "used by the Wan samplers is built")
        self.num_train_timesteps, self.solver_order, self.shift = num_train_timesteps, solver_order, shift
        self.solver_type, self.lower_order_final = solver_type, lower_order_final
        self.disable_corrector = list(disable_corrector)
        alphas = np.linspace(1, 1 / num_train_timesteps, num_train_timesteps)[::-1].copy()
        sigmas = torch.from_numpy(1.0 - alphas).to(dtype=torch.float32)
        sigmas = shift * sigmas / (1 + (shift - 1) * sigmas)
        self.sigmas = sigmas
        self.timesteps = sigmas * num_train_timesteps
        self.sigma_min = self.sigmas[-1].item()
        self.sigma_max = self.sigmas[0].item()
        self.num_inference_steps = None
        self._reset()

    def _reset(self):
        self.model_outputs = [None] * self.solver_order
        self.lower_order_nums = 0
        self.last_sample = None
        self._step_index = None
        self.this_order = None

    def set_timesteps(self, num_inference_steps, device=None, sigmas=None, mu=None, shift=None):
        """fm_solvers_unipc.py:162-229 (static shift, final sigma 0)."""
        if sigmas is None:
            sigmas = np.linspace(self.sigma_max, self.sigma_min, num_inference_steps + 1).copy()[:-1]
        shift = self.shift if shift is None else shift
        sigmas = shift * sigmas / (1 + (shift - 1) * sigmas)
        timesteps = sigmas * self.num_train_timesteps
        self.sigmas = torch.from_numpy(np.concatenate([sigmas, [0]]).astype(np.float32))
        self.timesteps = torch.from_numpy(timesteps).to(device=device, dtype=torch.int64)
        self.num_inference_steps = len(timesteps)
        self._reset()

    @property
    def step_index(self):
        return self._step_index

    # ------------------------------------------------------------------ coefficients (host, fp32)
    def _base(self, sigma_t, sigma_s0):
        alpha_t = 1 - sigma_t
        h = _lam(sigma_t) - _lam(sigma_s0)
        hh = -h
        h_phi_1 = torch.expm1(hh)
        B_h = hh if self.solver_type == "bh1" else torch.expm1(hh)
        return alpha_t, h, hh, h_phi_1, B_h

    def _launch(self, out, x, m0, m1, mt, mode, c):
        coef = (ctypes.c_float * 6)(*[float(v) for v in c])
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        _lib.check(_lib.load().vs_unipc_update(out.data_ptr(), ptr(x), ptr(m0), ptr(m1), ptr(mt), out.numel(), mode,
                                               coef, torch.cuda.current_stream(out.device).cuda_stream))
        return out

    def _uni_p(self, sample, order):
        """multistep_uni_p_bh_update (:352-486)."""
        i = self._step_index
        sigma_t, sigma_s0 = self.sigmas[i + 1], self.sigmas[i]
        alpha_t, h, hh, h_phi_1, B_h = self._base(sigma_t, sigma_s0)
        c1, c2, c3 = sigma_t / sigma_s0, alpha_t * h_phi_1, alpha_t * B_h
        m0 = self.model_outputs[-1]
        out = torch.empty_like(sample)
        if order == 1:
            return self._launch(out, sample, m0, None, None, 1, (c1, c2, c3, 0, 0, 1))
        if order != 2:
            raise NotImplementedError("UniP order > 2")
        rk = (_lam(self.sigmas[i - 1]) - _lam(sigma_s0)) / h
        return self._launch(out, sample, m0, self.model_outputs[-2], None, 2, (c1, c2, c3, 0.5, 0, rk))

    def _uni_c(self, this_model_output, last_sample, this_sample, order):
        """multistep_uni_c_bh_update (:488-628)."""
        i = self._step_index
        sigma_t, sigma_s0 = self.sigmas[i], self.sigmas[i - 1]
        alpha_t, h, hh, h_phi_1, B_h = self._base(sigma_t, sigma_s0)
        c1, c2, c3 = sigma_t / sigma_s0, alpha_t * h_phi_1, alpha_t * B_h
        m0 = self.model_outputs[-1]
        out = torch.empty_like(this_sample)
        if order == 1:
            return self._launch(out, last_sample, m0, None, this_model_output, 3, (c1, c2, c3, 0, 0.5, 1))
        if order != 2:
            raise NotImplementedError("UniC order > 2")
        rk = (_lam(self.sigmas[i - 2]) - _lam(sigma_s0)) / h
        rks = torch.tensor([rk, 1.0])
        R, b = [], []
        h_phi_k = h_phi_1 / hh - 1
        factorial_i = 1
        for k in range(1, order + 1):
            R.append(torch.pow(rks, k - 1))
            b.append(h_phi_k * factorial_i / B_h)
            factorial_i *= k + 1
            h_phi_k = h_phi_k / hh - 1 / factorial_i
        rhos_c = torch.linalg.solve(torch.stack(R), torch.tensor(b)).to(torch.float32)
        return self._launch(out, last_sample, m0, self.model_outputs[-2], this_model_output, 4,
                            (c1, c2, c3, rhos_c[0], rhos_c[1], rk))

    # ------------------------------------------------------------------ step (:657-741)
    def index_for_timestep(self, timestep):
        indices = (self.timesteps == timestep).nonzero()
        return indices[1 if len(indices) > 1 else 0].item()

    def step(self, model_output, timestep, sample, return_dict=False, generator=None):
        """model_output, sample: fp32 device tensors of one shape.  Returns (prev_sample,)."""
        if self.num_inference_steps is None:
            raise ValueError("call set_timesteps first")
        if model_output.dtype != torch.float32 or sample.dtype != torch.float32:
            raise ValueError("UniPC state is fp32: pass fp32 model_output / sample")
        model_output, sample = model_output.contiguous(), sample.contiguous()
        if self._step_index is None:
            t = timestep.cpu() if isinstance(timestep, torch.Tensor) else timestep
            self._step_index = self.index_for_timestep(t)
        i = self._step_index
        use_corrector = i > 0 and (i - 1) not in self.disable_corrector and self.last_sample is not None
        conv = self._launch(torch.empty_like(sample), sample, None, None, model_output, 0,
                            (self.sigmas[i], 0, 0, 0, 0, 1))
        if use_corrector:
            sample = self._uni_c(conv, self.last_sample, sample, self.this_order)
        for k in range(self.solver_order - 1):
            self.model_outputs[k] = self.model_outputs[k + 1]
        self.model_outputs[-1] = conv
        this_order = min(self.solver_order, len(self.timesteps) - i) if self.lower_order_final else self.solver_order
        self.this_order = min(this_order, self.lower_order_nums + 1)
        self.last_sample = sample
        prev = self._uni_p(sample, self.this_order)
        if self.lower_order_nums < self.solver_order:
            self.lower_order_nums += 1
        self._step_index += 1
        return (prev,)


def cast(src, dst):
    """fp32 <-> bf16 elementwise (vs_cast)."""
    to_bf16 = dst.dtype == torch.bfloat16
    _lib.check(_lib.load().vs_cast(src.data_ptr(), dst.data_ptr(), src.numel(), int(to_bf16),
                                   torch.cuda.current_stream(src.device).cuda_stream))
    return dst

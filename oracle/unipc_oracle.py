"""TEST INFRASTRUCTURE ONLY -- CPU restatement of FlowUniPCMultistepScheduler
(denoising_enhancing/wan/utils/fm_solvers_unipc.py:22-741) for flow prediction, predict-x0, bh2,
static shift, final sigma 0 -- the configuration of the Wan samplers (config 5's 4-step UniPC).
All tensor math in fp32 torch ops in the reference's order.  Parity status: numerics unpinned (no
reference vectors); the sigma/timestep tables follow the reference code line by line."""
import numpy as np
import torch


class UniPCOracle:
    def __init__(self, num_train_timesteps=1000, solver_order=2, shift=1.0, lower_order_final=True,
                 disable_corrector=()):
        self.N, self.order, self.shift = num_train_timesteps, solver_order, shift        # :79-97
        self.lower_order_final, self.disable_corrector = lower_order_final, list(disable_corrector)
        alphas = np.linspace(1, 1 / num_train_timesteps, num_train_timesteps)[::-1].copy()   # :109-120
        sigmas = torch.from_numpy(1.0 - alphas).to(dtype=torch.float32)
        sigmas = shift * sigmas / (1 + (shift - 1) * sigmas)
        self.sigma_min, self.sigma_max = sigmas[-1].item(), sigmas[0].item()

    def set_timesteps(self, n, shift=None):                                                 # :162-229
        sigmas = np.linspace(self.sigma_max, self.sigma_min, n + 1).copy()[:-1]
        shift = self.shift if shift is None else shift
        sigmas = shift * sigmas / (1 + (shift - 1) * sigmas)
        timesteps = sigmas * self.N
        self.sigmas = torch.from_numpy(np.concatenate([sigmas, [0]]).astype(np.float32))
        self.timesteps = torch.from_numpy(timesteps).to(dtype=torch.int64)
        self.model_outputs = [None] * self.order
        self.lower_order_nums, self.last_sample, self.step_index, self.this_order = 0, None, None, None

    @staticmethod
    def _lam(s):
        return torch.log(1 - s) - torch.log(s)

    def _coefs(self, sigma_t, sigma_s0, order, prev_si):
        alpha_t = 1 - sigma_t
        h = self._lam(sigma_t) - self._lam(sigma_s0)
        hh = -h
        h_phi_1 = torch.expm1(hh)
        B_h = torch.expm1(hh)
        rks = []
        if order == 2:
            rks.append((self._lam(self.sigmas[prev_si]) - self._lam(sigma_s0)) / h)
        rks.append(1.0)
        rks = torch.tensor(rks)
        R, b, h_phi_k, f = [], [], h_phi_1 / hh - 1, 1
        for i in range(1, order + 1):
            R.append(torch.pow(rks, i - 1))
            b.append(h_phi_k * f / B_h)
            f *= i + 1
            h_phi_k = h_phi_k / hh - 1 / f
        return alpha_t, h_phi_1, B_h, rks, torch.stack(R), torch.tensor(b)

    def _uni_p(self, x, order):                                                             # :352-486
        i = self.step_index
        sigma_t, sigma_s0 = self.sigmas[i + 1], self.sigmas[i]
        alpha_t, h_phi_1, B_h, rks, R, b = self._coefs(sigma_t, sigma_s0, order, i - 1)
        m0 = self.model_outputs[-1]
        x_t_ = sigma_t / sigma_s0 * x - alpha_t * h_phi_1 * m0
        if order == 2:
            D1 = (self.model_outputs[-2] - m0) / rks[0]
            pred_res = torch.einsum("k,bkc...->bc...", torch.tensor([0.5]), torch.stack([D1], dim=1))
            return x_t_ - alpha_t * B_h * pred_res
        return x_t_

    def _uni_c(self, model_t, x, order):                                                    # :488-628
        i = self.step_index
        sigma_t, sigma_s0 = self.sigmas[i], self.sigmas[i - 1]
        alpha_t, h_phi_1, B_h, rks, R, b = self._coefs(sigma_t, sigma_s0, order, i - 2)
        m0 = self.model_outputs[-1]
        rhos_c = torch.tensor([0.5]) if order == 1 else torch.linalg.solve(R, b).to(torch.float32)
        x_t_ = sigma_t / sigma_s0 * x - alpha_t * h_phi_1 * m0
        corr_res = 0
        if order == 2:
            D1 = (self.model_outputs[-2] - m0) / rks[0]
            corr_res = torch.einsum("k,bkc...->bc...", rhos_c[:-1], torch.stack([D1], dim=1))
        return x_t_ - alpha_t * B_h * (corr_res + rhos_c[-1] * (model_t - m0))

    def step(self, model_output, timestep, sample):                                         # :657-741
        if self.step_index is None:
            idx = (self.timesteps == timestep).nonzero()
            self.step_index = idx[1 if len(idx) > 1 else 0].item()
        i = self.step_index
        use_corrector = i > 0 and (i - 1) not in self.disable_corrector and self.last_sample is not None
        conv = sample - self.sigmas[i] * model_output                                       # :317-323
        if use_corrector:
            sample = self._uni_c(conv, self.last_sample, self.this_order)
        for k in range(self.order - 1):
            self.model_outputs[k] = self.model_outputs[k + 1]
        self.model_outputs[-1] = conv
        this_order = min(self.order, len(self.timesteps) - i) if self.lower_order_final else self.order
        self.this_order = min(this_order, self.lower_order_nums + 1)
        self.last_sample = sample
        prev = self._uni_p(sample, self.this_order)
        if self.lower_order_nums < self.order:
            self.lower_order_nums += 1
        self.step_index += 1
        return prev

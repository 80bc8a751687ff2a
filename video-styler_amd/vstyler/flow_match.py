"""FlowMatchScheduler with the reference's API (diffsynth/schedulers/flow_match.py:5-125).

The sigma/timestep table is host data (as in the reference); the Euler update itself runs on the
GPU through vs_cfg_euler.  `step()` keeps the reference signature for drop-in use and routes the
bf16 update through the same kernel.
"""
import math

import torch

from . import kernels as K


class FlowMatchScheduler:
    def __init__(self, num_inference_steps=100, num_train_timesteps=1000, shift=3.0, sigma_max=1.0,
                 sigma_min=0.003 / 1.002, inverse_timesteps=False, extra_one_step=False, reverse_sigmas=False,
                 exponential_shift=False, exponential_shift_mu=None, shift_terminal=None):
        self.num_train_timesteps = num_train_timesteps
        self.shift = shift
        self.sigma_max = sigma_max
        self.sigma_min = sigma_min
        self.inverse_timesteps = inverse_timesteps
        self.extra_one_step = extra_one_step
        self.reverse_sigmas = reverse_sigmas
        self.exponential_shift = exponential_shift
        self.exponential_shift_mu = exponential_shift_mu
        self.shift_terminal = shift_terminal
        self.set_timesteps(num_inference_steps)

    def set_timesteps(self, num_inference_steps=100, denoising_strength=1.0, training=False, shift=None,
                      dynamic_shift_len=None, exponential_shift_mu=None):
        """flow_match.py:34-69."""
        if shift is not None:
            self.shift = shift
        sigma_start = self.sigma_min + (self.sigma_max - self.sigma_min) * denoising_strength
        if self.extra_one_step:
            self.sigmas = torch.linspace(sigma_start, self.sigma_min, num_inference_steps + 1)[:-1]
        else:
            self.sigmas = torch.linspace(sigma_start, self.sigma_min, num_inference_steps)
        if self.inverse_timesteps:
            self.sigmas = torch.flip(self.sigmas, dims=[0])
        if self.exponential_shift:
            mu = exponential_shift_mu if exponential_shift_mu is not None else (
                self.calculate_shift(dynamic_shift_len) if dynamic_shift_len is not None else self.exponential_shift_mu)
            self.sigmas = math.exp(mu) / (math.exp(mu) + (1 / self.sigmas - 1))
        else:
            self.sigmas = self.shift * self.sigmas / (1 + (self.shift - 1) * self.sigmas)
        if self.shift_terminal is not None:
            one_minus_z = 1 - self.sigmas
            scale_factor = one_minus_z[-1] / (1 - self.shift_terminal)
            self.sigmas = 1 - (one_minus_z / scale_factor)
        if self.reverse_sigmas:
            self.sigmas = 1 - self.sigmas
        self.timesteps = self.sigmas * self.num_train_timesteps
        self.training = bool(training)

    def _index(self, timestep):
        if isinstance(timestep, torch.Tensor):
            timestep = timestep.detach().float().cpu()
        return int(torch.argmin((self.timesteps - timestep).abs()))

    def delta(self, step_index, to_final=False):
        """fp32 (sigma_{i+1} - sigma_i) of flow_match.py:75-81 as a python float."""
        sigma = self.sigmas[step_index]
        if to_final or step_index + 1 >= len(self.timesteps):
            sigma_ = 1 if (self.inverse_timesteps or self.reverse_sigmas) else 0
        else:
            sigma_ = self.sigmas[step_index + 1]
        return float(sigma_ - sigma)

    def step(self, model_output, timestep, sample, to_final=False, **kwargs):
        """flow_match.py:72-82 (returns a new bf16 tensor; computed by vs_cfg_euler)."""
        out = sample.contiguous().clone()
        K.cfg_euler(model_output.contiguous(), None, out, 1.0, self.delta(self._index(timestep), to_final))
        return out

    def add_noise(self, original_samples, noise, timestep):
        sigma = self.sigmas[self._index(timestep)]
        return (1 - sigma) * original_samples + sigma * noise

    def training_target(self, sample, noise, timestep):
        return noise - sample

    def calculate_shift(self, image_seq_len, base_seq_len=256, max_seq_len=8192, base_shift=0.5, max_shift=0.9):
        m = (max_shift - base_shift) / (max_seq_len - base_seq_len)
        b = base_shift - m * base_seq_len
        return image_seq_len * m + b

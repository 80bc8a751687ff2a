"""TeaCache step skipping (reference: class TeaCache, diffsynth/pipelines/wan_video_new.py:1154-1203;
unit WanVideoUnit_TeaCache :936-947; use in model_fn_wan_video :1398-1402,1418-1419,1455-1456).

Per step, the relative L1 change of the modulation input t_mod is mapped through a per-model
polynomial and accumulated; while the sum stays below the threshold the DiT blocks (and VACE) are
skipped and the hidden states advanced by the residual of the last computed step.  The decision
uses the reference's arithmetic on the bf16 t_mod (bf16 abs/mean/div, then numpy poly1d in
float64); the residual store/update are the bf16 adds of the reference, done by vs_axpy on the GPU.

Differences kept deliberately: the reference evaluates the VACE branch even on skipped steps
(its hints are then unused); this build skips it -- the output is identical.  Under CFG the
reference keeps one TeaCache per prompt (same t_mod -> same decisions); this build keeps one
for the batch-2 forward, whose residual rows are the two per-prompt residuals."""
import numpy as np
import torch

from . import kernels as K

COEFFICIENTS = {   # wan_video_new.py:1164-1169
    "Wan2.1-T2V-1.3B": [-5.21862437e+04, 9.23041404e+03, -5.28275948e+02, 1.36987616e+01, -4.99875664e-02],
    "Wan2.1-T2V-14B": [-3.03318725e+05, 4.90537029e+04, -2.65530556e+03, 5.87365115e+01, -3.15583525e-01],
    "Wan2.1-I2V-14B-480P": [2.57151496e+05, -3.54229917e+04, 1.40286849e+03, -1.35890334e+01, 1.32517977e-01],
    "Wan2.1-I2V-14B-720P": [8.10705460e+03, 2.13393892e+03, -3.72934672e+02, 1.66203073e+01, -4.17769401e-02],
}


def rel_l1(t_mod, prev):
    """((t_mod - prev).abs().mean() / prev.abs().mean()).item() in bf16, as :1178."""
    a = t_mod.detach().to("cpu")
    b = prev.detach().to("cpu")
    return ((a - b).abs().mean() / b.abs().mean()).item()


class TeaCache:
    def __init__(self, num_inference_steps, rel_l1_thresh, model_id):
        if model_id not in COEFFICIENTS:
            raise ValueError(f"{model_id} is not a supported TeaCache model id. Please choose a valid model id in "
                             f"({', '.join(COEFFICIENTS)}).")
        self.num_inference_steps = num_inference_steps
        self.rel_l1_thresh = rel_l1_thresh
        self.coefficients = COEFFICIENTS[model_id]
        self.step = 0
        self.accumulated_rel_l1_distance = 0
        self.previous_modulated_input = None
        self.previous_hidden_states = None
        self.previous_residual = None
        self.decisions = []          # True = computed, False = skipped (for tests / logs)

    def check(self, dit, x, t_mod):
        """:1173-1192 -> True when the blocks are to be SKIPPED.  t_mod: (1, 6, D) bf16 (one
        prompt's row; all CFG rows are identical)."""
        modulated_inp = t_mod.clone()
        if self.step == 0 or self.step == self.num_inference_steps - 1:
            should_calc = True
            self.accumulated_rel_l1_distance = 0
        else:
            self.accumulated_rel_l1_distance += np.poly1d(self.coefficients)(
                rel_l1(modulated_inp, self.previous_modulated_input))
            if self.accumulated_rel_l1_distance < self.rel_l1_thresh:
                should_calc = False
            else:
                should_calc = True
                self.accumulated_rel_l1_distance = 0
        self.previous_modulated_input = modulated_inp
        self.step += 1
        if self.step == self.num_inference_steps:
            self.step = 0
        self.decisions.append(should_calc)
        return not should_calc

    def begin(self, x):
        """Called on a computed step before the blocks (:1192-1193): keep the input hidden states."""
        if self.previous_hidden_states is None or self.previous_hidden_states.shape != x.shape:
            self.previous_hidden_states = torch.empty_like(x)
        self.previous_hidden_states.copy_(x)

    def store(self, x):
        """:1195-1197: residual = bf16(x - previous_hidden_states)."""
        if self.previous_residual is None or self.previous_residual.shape != x.shape:
            self.previous_residual = torch.empty_like(x)
        self.previous_residual.copy_(x)
        K.axpy(self.previous_residual, self.previous_hidden_states, -1.0)

    def update(self, x):
        """:1199-1201: x = bf16(x + residual), in place."""
        K.axpy(x, self.previous_residual, 1.0)
        return x

"""Restatement of diffusers' ``DDIMScheduler`` (golden generation only).

Defaults and arithmetic as the reference uses them: constructed at
transfuser_model_v2.py:447-451 (``scaled_linear``, ``prediction_type='sample'``,
``clip_sample=True`` and ``set_alpha_to_one=True`` by default), ``set_timesteps`` at
:584, ``add_noise`` at :595-597 and ``step`` (eta = 0) at :634-636. All schedule
arithmetic stays in float32 tensors, as diffusers does.
"""
import numpy as np
import torch


class _Out:
    def __init__(self, prev_sample, pred_original_sample):
        self.prev_sample = prev_sample
        self.pred_original_sample = pred_original_sample


class DDIMScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.0001, beta_end=0.02,
                 beta_schedule="linear", clip_sample=True, set_alpha_to_one=True,
                 steps_offset=0, prediction_type="epsilon", clip_sample_range=1.0):
        self.num_train_timesteps = num_train_timesteps
        if beta_schedule == "linear":
            self.betas = torch.linspace(beta_start, beta_end, num_train_timesteps,
                                        dtype=torch.float32)
        elif beta_schedule == "scaled_linear":
            self.betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5,
                                        num_train_timesteps, dtype=torch.float32) ** 2
        else:
            raise NotImplementedError(beta_schedule)
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.clip_sample = clip_sample
        self.clip_sample_range = clip_sample_range
        self.prediction_type = prediction_type
        self.steps_offset = steps_offset
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, num_train_timesteps)[::-1].copy().astype(np.int64))

    def set_timesteps(self, num_inference_steps, device=None):
        self.num_inference_steps = num_inference_steps
        step_ratio = self.num_train_timesteps // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * step_ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = torch.from_numpy(ts + self.steps_offset).to(device)

    def add_noise(self, original_samples, noise, timesteps):
        ac = self.alphas_cumprod.to(device=original_samples.device, dtype=original_samples.dtype)
        timesteps = timesteps.to(original_samples.device)
        sa = (ac[timesteps] ** 0.5).flatten()
        while sa.dim() < original_samples.dim():
            sa = sa.unsqueeze(-1)
        s1 = ((1 - ac[timesteps]) ** 0.5).flatten()
        while s1.dim() < original_samples.dim():
            s1 = s1.unsqueeze(-1)
        return sa * original_samples + s1 * noise

    def step(self, model_output, timestep, sample, eta=0.0, use_clipped_model_output=False,
             generator=None, variance_noise=None, return_dict=True):
        prev_t = timestep - self.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[timestep]
        a_prev = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.final_alpha_cumprod
        b_t = 1 - a_t
        if self.prediction_type == "sample":
            x0 = model_output
            eps = (sample - a_t ** 0.5 * x0) / b_t ** 0.5
        elif self.prediction_type == "epsilon":
            x0 = (sample - b_t ** 0.5 * model_output) / a_t ** 0.5
            eps = model_output
        else:
            raise NotImplementedError(self.prediction_type)
        if self.clip_sample:
            x0 = x0.clamp(-self.clip_sample_range, self.clip_sample_range)
        b_prev = 1 - a_prev
        variance = (b_prev / b_t) * (1 - a_t / a_prev)
        std = eta * variance ** 0.5
        if use_clipped_model_output:
            eps = (sample - a_t ** 0.5 * x0) / b_t ** 0.5
        direction = (1 - a_prev - std ** 2) ** 0.5 * eps
        prev = a_prev ** 0.5 * x0 + direction
        return _Out(prev, x0)

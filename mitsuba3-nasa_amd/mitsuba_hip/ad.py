"""mi.ad optimizers (src/python/python/ad/optimizers.py).

The inverse-rendering loop around the hot path:

    opt = mi.ad.Adam(lr=0.05)
    opt['white.reflectance.value'] = params['white.reflectance.value']
    params.update(opt)
    for it in range(n):
        img = mi.render(scene, params, seed=it)
        loss = ((img - ref) ** 2).mean()
        loss.backward()            # -> render_backward (PRB) on the device
        opt.step()
        opt[k] = opt[k].clamp(0, 1)
        params.update(opt)

Parameters are device tensors with `requires_grad`, the torch stand-in for
Dr.Jit's `enable_grad`; the update rules, bias correction, `mask_updates`,
`uniform` (UniformAdam) and the SGD-momentum step (which applies the state of
the previous iteration, optimizers.py:160-168) follow the reference exactly.
All arithmetic is float32 on the parameter's device.
"""
from __future__ import annotations

import math
from collections import defaultdict


def _torch():
    import torch
    return torch


class Optimizer:
    """optimizers.py:6-104."""

    def __init__(self, lr, params=None):
        self.lr = defaultdict(lambda: self.lr_default)
        self.set_learning_rate(lr)
        self.variables = {}
        self.state = {}
        if params is not None:
            for k, v in params.items():
                self.__setitem__(k, v)

    def __contains__(self, key):
        return key in self.variables

    def __getitem__(self, key):
        return self.variables[key]

    def __setitem__(self, key, value):
        torch = _torch()
        if not (torch.is_tensor(value) and value.is_floating_point()):
            raise Exception("Optimizer.__setitem__(): value should be differentiable!")
        needs_reset = key not in self.variables or self.variables[key].shape != value.shape
        self.variables[key] = value.detach().clone().requires_grad_(True)
        if needs_reset:
            self.reset(key)

    def __delitem__(self, key):
        del self.variables[key]

    def __len__(self):
        return len(self.variables)

    def keys(self):
        return self.variables.keys()

    def items(self):
        return list(self.variables.items())

    def set_learning_rate(self, lr):
        if isinstance(lr, (float, int)):
            self.lr_default = float(lr)
        elif isinstance(lr, dict):
            for k, v in lr.items():
                self.lr[k] = float(v)
        else:
            raise Exception("Optimizer.set_learning_rate(): value should be a float or a dict!")

    def reset(self, key):
        pass

    def _commit(self, key, value):
        self.variables[key] = value.detach().requires_grad_(True)


class SGD(Optimizer):
    """optimizers.py:107-199."""

    def __init__(self, lr, momentum=0, mask_updates=False, params=None):
        assert 0 <= momentum < 1 and lr > 0
        self.momentum = momentum
        self.mask_updates = mask_updates
        super().__init__(lr, params)

    def step(self):
        torch = _torch()
        for k, p in list(self.variables.items()):
            g = p.grad
            if g is None or g.numel() == 0:
                continue
            lr = torch.tensor(self.lr[k], dtype=p.dtype, device=p.device)
            if self.momentum != 0:
                if self.state[k].shape != g.shape:
                    self.reset(k)
                nxt = self.momentum * self.state[k] + g
                step = lr * self.state[k]          # the previous state, as the reference
                if self.mask_updates:
                    nz = g != 0
                    nxt = torch.where(nz, nxt, self.state[k])
                    step = torch.where(nz, step, torch.zeros_like(step))
                self.state[k] = nxt
                value = p.detach() - step
            else:
                value = p.detach() - lr * g
            self._commit(k, value)

    def reset(self, key):
        torch = _torch()
        if self.momentum == 0:
            return
        self.state[key] = torch.zeros_like(self.variables[key].detach())

    def __repr__(self):
        return (f"SGD[\n  variables = {list(self.keys())},\n  lr = {dict(self.lr, default=self.lr_default)},\n"
                f"  momentum = {self.momentum:.2g}\n]")


class Adam(Optimizer):
    """optimizers.py:204-321."""

    def __init__(self, lr, beta_1=0.9, beta_2=0.999, epsilon=1e-8, mask_updates=False, uniform=False,
                 params=None):
        assert 0 <= beta_1 < 1 and 0 <= beta_2 < 1 and epsilon > 0
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon
        self.mask_updates, self.uniform = mask_updates, uniform
        self.t = defaultdict(lambda: 0)
        super().__init__(lr, params)

    def step(self):
        torch = _torch()
        for k, p in list(self.variables.items()):
            self.t[k] += 1
            lr_scale = math.sqrt(1 - self.beta_2 ** self.t[k]) / (1 - self.beta_1 ** self.t[k])
            f32 = dict(dtype=torch.float32, device=p.device)
            lr_t = torch.tensor(self.lr[k], **f32) * torch.tensor(lr_scale, **f32)
            g = p.grad
            if g is None or g.numel() == 0:
                continue
            if self.state[k][0].shape != g.shape:
                self.reset(k)
            m_tp, v_tp = self.state[k]
            m_t = self.beta_1 * m_tp + (1 - self.beta_1) * g
            v_t = self.beta_2 * v_tp + (1 - self.beta_2) * g * g
            if self.mask_updates:
                nz = g != 0
                m_t = torch.where(nz, m_t, m_tp)
                v_t = torch.where(nz, v_t, v_tp)
            self.state[k] = (m_t, v_t)
            if self.uniform:
                step = lr_t * m_t / (torch.sqrt(v_t.max()) + self.epsilon)
            else:
                step = lr_t * m_t / (torch.sqrt(v_t) + self.epsilon)
            if self.mask_updates:
                step = torch.where(nz, step, torch.zeros_like(step))
            self._commit(k, p.detach() - step)

    def reset(self, key):
        torch = _torch()
        p = self.variables[key].detach()
        self.state[key] = (torch.zeros_like(p), torch.zeros_like(p))
        self.t[key] = 0

    def __repr__(self):
        return (f"Adam[\n  variables = {list(self.keys())},\n  lr = {dict(self.lr, default=self.lr_default)},\n"
                f"  betas = ({self.beta_1:g}, {self.beta_2:g}),\n  eps = {self.epsilon:g}\n]")

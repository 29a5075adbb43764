"""``paddle.incubate.optimizer`` (reference `incubate/optimizer/{lookahead,modelaverage}.py`,
`functional/{bfgs,lbfgs}.py`): LookAhead, ModelAverage, minimize_bfgs, minimize_lbfgs."""
from __future__ import annotations

import torch

__all__ = ["LookAhead", "ModelAverage"]


class LookAhead:
    """Wraps an inner optimizer: every ``k`` steps the slow weights move ``alpha`` of the way to
    the fast weights and the fast weights are reset to them (Zhang et al., 2019)."""

    def __init__(self, inner_optimizer, alpha=0.5, k=5, name=None):
        assert 0.0 <= alpha <= 1.0 and k >= 1
        self.inner_optimizer, self.alpha, self.k = inner_optimizer, alpha, k
        self._params = [p for p in inner_optimizer._parameter_list]
        self._slow = [p.detach().clone() for p in self._params]
        self._step = 0

    @torch.no_grad()
    def step(self):
        self.inner_optimizer.step()
        self._step += 1
        if self._step % self.k == 0:
            for p, s in zip(self._params, self._slow):
                s.add_(p.detach() - s, alpha=self.alpha)
                p.copy_(s)

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.step()

    def clear_grad(self, set_to_zero=True):
        self.inner_optimizer.clear_grad(set_to_zero)

    def state_dict(self):
        return {"inner": self.inner_optimizer.state_dict(), "slow": self._slow, "step": self._step}

    def set_state_dict(self, sd):
        self.inner_optimizer.set_state_dict(sd["inner"])
        for s, v in zip(self._slow, sd["slow"]):
            s.copy_(v)
        self._step = sd["step"]


class ModelAverage:
    """Running average of the parameters over a sliding window (``average_window_rate`` of the
    steps, clamped to [min_average_window, max_average_window]); ``apply()`` swaps the averages in
    (context manager, restored on exit unless ``need_restore=False``)."""

    def __init__(self, average_window_rate, parameters=None, min_average_window=10000,
                 max_average_window=10000, name=None):
        self.rate, self.min_w, self.max_w = average_window_rate, min_average_window, max_average_window
        self._params = [p for p in (parameters or [])]
        self._sum = [torch.zeros_like(p, dtype=torch.float32) for p in self._params]
        self._n = 0
        self._steps = 0
        self._backup = None

    @torch.no_grad()
    def step(self):
        self._steps += 1
        window = max(self.min_w, min(self.max_w, int(self._steps * self.rate)))
        if self._n >= window:  # restart the window (reference: sum_1/sum_2/sum_3 rotation)
            for s in self._sum:
                s.zero_()
            self._n = 0
        for s, p in zip(self._sum, self._params):
            s.add_(p.detach().float())
        self._n += 1

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()

    class _Apply:
        def __init__(self, ma, need_restore):
            self.ma, self.need_restore = ma, need_restore

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            if self.need_restore:
                self.ma.restore()

    @torch.no_grad()
    def apply(self, executor=None, need_restore=True):
        self._backup = [p.detach().clone() for p in self._params]
        if self._n:
            for p, s in zip(self._params, self._sum):
                p.copy_((s / self._n).to(p.dtype))
        return ModelAverage._Apply(self, need_restore)

    @torch.no_grad()
    def restore(self, executor=None):
        if self._backup is not None:
            for p, b in zip(self._params, self._backup):
                p.copy_(b)
            self._backup = None


def _minimize(objective_func, initial_position, max_iters, tolerance_grad, tolerance_change,
              history_size, line_search_fn, dtype):
    x = initial_position.detach().clone().to(getattr(torch, dtype) if isinstance(dtype, str) else dtype)
    x.requires_grad_(True)
    opt = torch.optim.LBFGS([x], max_iter=max_iters, tolerance_grad=tolerance_grad,
                            tolerance_change=tolerance_change, history_size=history_size,
                            line_search_fn="strong_wolfe" if line_search_fn else None)
    calls = {"n": 0}

    def closure():
        opt.zero_grad()
        f = objective_func(x)
        f.backward()
        calls["n"] += 1
        return f
    opt.step(closure)
    f = objective_func(x)
    g, = torch.autograd.grad(f, x)
    converged = bool(g.abs().max() <= tolerance_grad)
    return converged, calls["n"], x.detach(), f.detach(), g.detach()


def minimize_lbfgs(objective_func, initial_position, history_size=100, max_iters=50,
                   tolerance_grad=1e-8, tolerance_change=1e-8, initial_inverse_hessian_estimate=None,
                   line_search_fn="strong_wolfe", max_line_search_iters=50,
                   initial_step_length=1.0, dtype="float32", name=None):
    """Returns (is_converge, num_func_calls, position, objective_value, objective_gradient)."""
    return _minimize(objective_func, initial_position, max_iters, tolerance_grad, tolerance_change,
                     history_size, line_search_fn, dtype)


def minimize_bfgs(objective_func, initial_position, max_iters=50, tolerance_grad=1e-7,
                  tolerance_change=1e-9, initial_inverse_hessian_estimate=None,
                  line_search_fn="strong_wolfe", max_line_search_iters=50, initial_step_length=1.0,
                  dtype="float32", name=None):
    """Full-memory quasi-Newton (history = max_iters) with strong-Wolfe line search."""
    return _minimize(objective_func, initial_position, max_iters, tolerance_grad, tolerance_change,
                     max(1, max_iters), line_search_fn, dtype)


class functional:  # noqa: N801  (namespace: paddle.incubate.optimizer.functional)
    minimize_bfgs = staticmethod(minimize_bfgs)
    minimize_lbfgs = staticmethod(minimize_lbfgs)

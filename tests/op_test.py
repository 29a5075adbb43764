"""OpTest harness (the role of reference `fluid/tests/unittests/op_test.py`): an op case declares
numpy ``inputs``, ``attrs`` and the numpy-computed ``outputs`` it expects; ``check_output`` runs the
framework op and compares, ``check_grad`` compares the framework's analytic gradient (autograd
through our kernels / compositions) with a central finite difference taken in float64.

The numeric gradient is of ``sum(out * w)`` for a fixed random ``w`` (like the reference's
``user_defined_grad_outputs`` default of a random upstream gradient), so a wrong-sign or
wrong-layout gradient cannot hide behind a uniform upstream gradient.
"""
from __future__ import annotations

import numpy as np
import torch


class OpTest:
    """Subclass and set ``op`` (callable taking tensors by keyword + attrs) in ``setUp``-like
    ``setup()``; ``inputs``: name → np.ndarray; ``attrs``: name → python value; ``outputs``:
    name → np.ndarray (single output: any name)."""

    op = None
    inputs: dict = {}
    attrs: dict = {}
    outputs: dict = {}
    device = "cpu"
    dtype = np.float64

    def setup(self):  # pragma: no cover - overridden
        raise NotImplementedError

    # ------------------------------------------------------------------ helpers
    def _tensors(self, requires_grad=(), dtype=None):
        out = {}
        for k, v in self.inputs.items():
            if isinstance(v, np.ndarray):
                t = torch.from_numpy(np.ascontiguousarray(v))
                if t.is_floating_point() and dtype is not None:
                    t = t.to(dtype)
                t = t.to(self.device)
                if k in requires_grad:
                    t.requires_grad_(True)
                out[k] = t
            else:
                out[k] = v
        return out

    def _run(self, tensors):
        res = type(self).op(**tensors, **self.attrs)
        if isinstance(res, (list, tuple)):
            return list(res)
        return [res]

    # ------------------------------------------------------------------ checks
    def check_output(self, atol=1e-5, rtol=1e-5, dtype=None):
        self.setup()
        got = self._run(self._tensors(dtype=dtype))
        want = list(self.outputs.values())
        assert len(got) >= len(want), f"{len(got)} outputs, expected {len(want)}"
        for name, g, w in zip(self.outputs, got, want):
            g = g.detach().float().cpu().numpy() if g.is_floating_point() else g.detach().cpu().numpy()
            np.testing.assert_allclose(g, w, atol=atol, rtol=rtol, err_msg=f"output {name}")

    def check_grad(self, inputs_to_check, output_index=0, max_relative_error=1e-5, delta=1e-6,
                   no_grad_set=()):
        self.setup()
        rng = np.random.default_rng(1234)
        tensors = self._tensors(requires_grad=set(inputs_to_check), dtype=torch.float64)
        out = self._run(tensors)[output_index]
        w = torch.from_numpy(rng.standard_normal(tuple(out.shape))).to(out)
        (out * w).sum().backward()
        for name in inputs_to_check:
            analytic = tensors[name].grad.detach().cpu().numpy()
            base = self.inputs[name].astype(np.float64)
            numeric = np.zeros_like(base)
            flat = base.reshape(-1)
            for i in range(flat.size):
                orig = flat[i]
                vals = []
                for sgn in (1, -1):
                    flat[i] = orig + sgn * delta
                    t2 = self._tensors(dtype=torch.float64)
                    t2[name] = torch.from_numpy(base.copy()).to(self.device)
                    with torch.no_grad():
                        o = self._run(t2)[output_index]
                    vals.append(float((o * w).sum()))
                flat[i] = orig
                numeric.reshape(-1)[i] = (vals[0] - vals[1]) / (2 * delta)
            scale = np.maximum(np.abs(numeric), 1e-3)
            err = np.max(np.abs(analytic - numeric) / scale)
            assert err <= max_relative_error, \
                f"grad of {name}: max relative error {err:.3g} > {max_relative_error}"

"""LocalSGD, adaptive LocalSGD and DGC (`distributed/fleet/comm_optimizers.py`; reference
`fleet/meta_optimizers/localsgd_optimizer.py`, `dgc_optimizer.py`, `operators/dgc_op.h`,
`optimizers/dgc_momentum_op.h`) on 2 gloo ranks, each against a single-process simulation of the
same algorithm over the two ranks' data."""
import copy
import math

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd.distributed import fleet

from dist_utils import run_distributed


def _mlp(seed=0, hidden=16):
    torch.manual_seed(seed)
    return torch.nn.Sequential(paddle.nn.Linear(8, hidden), torch.nn.ReLU(), paddle.nn.Linear(hidden, 1))


def _data(rank, n, B=8):
    g = torch.Generator().manual_seed(100 + rank)
    return [(torch.randn(B, 8, generator=g), torch.randn(B, 1, generator=g)) for _ in range(n)]


def _params(m):
    return [p.detach().clone() for p in m.parameters()]


def _worker(rank, world, flags, nsteps, opt_kind, hidden):
    st = fleet.DistributedStrategy()
    for k, v in flags.items():
        setattr(st, k, v)
    fleet.init(is_collective=True, strategy=st)
    m = _mlp(hidden=hidden)
    model = fleet.distributed_model(m)
    assert model is m  # no gradient reducer: the optimizer owns the communication
    if opt_kind == "sgd":
        o = paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters())
    else:
        o = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=m.parameters())
    opt = fleet.distributed_optimizer(o)
    losses, ks = [], []
    for x, y in _data(rank, nsteps):
        loss = ((model(x) - y) ** 2).mean()
        opt.minimize(loss)
        opt.clear_grad()
        losses.append(float(loss.detach()))
        ks.append(getattr(opt, "k_steps", None))
    return _params(m), losses, ks


def _sim_localsgd(nsteps, k_steps, begin_step, world=2, adaptive=False):
    ms = [_mlp() for _ in range(world)]
    opts = [paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters()) for m in ms]
    data = [_data(r, nsteps) for r in range(world)]
    last, ks, lr0, loss0, k = 0, [], None, None, k_steps
    for s in range(1, nsteps + 1):
        losses = []
        for r in range(world):
            x, y = data[r][s - 1]
            loss = ((ms[r](x) - y) ** 2).mean()
            loss.backward()
            opts[r].step()
            opts[r].clear_grad()
            losses.append(float(loss))
        if adaptive and lr0 is None:
            lr0, loss0 = 0.1, sum(losses) / world
        comm = s <= begin_step or s - last == k
        if comm:
            with torch.no_grad():
                for ps in zip(*[m.parameters() for m in ms]):
                    avg = sum(p for p in ps) / world
                    for p in ps:
                        p.copy_(avg)
            last = s
            if adaptive and s > begin_step:
                avg_loss = sum(losses) / world
                k = min(max(math.ceil(math.sqrt(lr0 * avg_loss / (0.1 * loss0) * k_steps)), 1), 16)
        ks.append(k)
    return _params(ms[0]), ks


@pytest.mark.parametrize("k_steps,begin_step", [(2, 1), (3, 2)])
def test_localsgd_matches_simulation(k_steps, begin_step):
    n = 7
    res = run_distributed(_worker, 2, {"localsgd": True,
                                       "localsgd_configs": {"k_steps": k_steps, "begin_step": begin_step}},
                          n, "sgd", 16)
    ref, _ = _sim_localsgd(n, k_steps, begin_step)
    for a, b in zip(res[0][0], ref):  # the simulation follows rank 0 exactly
        torch.testing.assert_close(torch.as_tensor(a), b, rtol=1e-5, atol=1e-6)
    if n <= begin_step or (n - begin_step) % k_steps == 0:  # last step averaged: ranks agree
        for a, b in zip(res[0][0], res[1][0]):
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)


def test_adaptive_localsgd_interval_follows_loss():
    n = 8
    res = run_distributed(_worker, 2, {"adaptive_localsgd": True,
                                       "adaptive_localsgd_configs": {"init_k_steps": 2, "begin_step": 2}},
                          n, "sgd", 16)
    ref, ks = _sim_localsgd(n, 2, 2, adaptive=True)
    assert res[0][2] == ks and res[1][2] == ks
    for a, b in zip(res[0][0], ref):
        torch.testing.assert_close(torch.as_tensor(a), b, rtol=1e-5, atol=1e-6)


def _sim_dgc(nsteps, rampup_begin, sparsity, hidden, world=2, lr=0.05, mu=0.9):
    """Single-process DGC over the two ranks' gradients (dgc_op.h + dgc_momentum_op.h)."""
    ms = [_mlp(hidden=hidden) for _ in range(world)]
    data = [_data(r, nsteps) for r in range(world)]
    params = list(ms[0].parameters())
    u = [torch.zeros_like(p) for p in params]                       # shared velocity (all ranks agree before ramp)
    us = [[torch.zeros_like(p) for p in params] for _ in range(world)]
    vs = [[torch.zeros_like(p) for p in params] for _ in range(world)]
    for s in range(nsteps):
        grads = []
        for r in range(world):
            x, y = data[r][s]
            for p in ms[r].parameters():
                p.grad = None
            loss = ((ms[r](x) - y) ** 2).mean()
            loss.backward()
            grads.append([p.grad.clone() for p in ms[r].parameters()])
        with torch.no_grad():
            for i, p0 in enumerate(params):
                big = p0.numel() >= 16384
                if s >= rampup_begin and big:
                    k = max(1, int(p0.numel() * (1 - sparsity)))
                    G = torch.zeros(p0.numel())
                    for r in range(world):
                        us[r][i].mul_(mu).add_(grads[r][i])
                        vs[r][i].add_(us[r][i])
                        vf = vs[r][i].view(-1)
                        idx = torch.topk(vf.abs(), k, sorted=False).indices
                        G.index_add_(0, idx, vf[idx])
                        vf[idx] = 0
                        us[r][i].view(-1)[idx] = 0
                    for r in range(world):
                        list(ms[r].parameters())[i].sub_((lr * G / world).view_as(p0))
                else:
                    g = sum(grads[r][i] for r in range(world)) / world
                    for r in range(world):
                        us[r][i].mul_(mu).add_(g)
                        list(ms[r].parameters())[i].sub_(lr * us[r][i])
    return _params(ms[0]), _params(ms[1])


@pytest.mark.parametrize("sparsity,rampup_begin", [(0.0, 0), (0.9, 2)])
def test_dgc_matches_simulation(sparsity, rampup_begin):
    n, hidden = 5, 2048  # first Linear: 8 x 2048 = 16384 elements → compressed; others dense
    res = run_distributed(_worker, 2, {"dgc": True,
                                       "dgc_configs": {"rampup_begin_step": rampup_begin, "rampup_step": 1,
                                                       "sparsity": [sparsity]}},
                          n, "momentum", hidden)
    ref0, ref1 = _sim_dgc(n, rampup_begin, sparsity, hidden)
    for got, ref in ((res[0][0], ref0), (res[1][0], ref1)):
        for a, b in zip(got, ref):
            torch.testing.assert_close(torch.as_tensor(a), b, rtol=2e-4, atol=2e-6)
    # the compressed parameter stays identical on both ranks (every rank applies the same sum)
    np.testing.assert_allclose(res[0][0][0], res[1][0][0], rtol=0, atol=0)


def test_sparsity_ramp_and_exclusivity():
    from paddle_infer_amd.distributed.fleet.comm_optimizers import _sparsity_at
    sp = [0.75, 0.9375, 0.984375, 0.996, 0.999]
    assert [_sparsity_at(sp, s, 5) for s in range(7)] == [0.75, 0.9375, 0.984375, 0.996, 0.999, 0.999, 0.999]
    st = fleet.DistributedStrategy()
    st.dgc = True
    st.localsgd = True
    with pytest.raises(ValueError):
        fleet.init(is_collective=True, strategy=st)


def test_dgc_needs_momentum():
    from paddle_infer_amd.distributed.fleet.comm_optimizers import DGCMomentumOptimizer
    m = _mlp()
    with pytest.raises(TypeError):
        DGCMomentumOptimizer(paddle.optimizer.Adam(parameters=m.parameters()))

"""Static-graph Fleet meta-optimizers as Program rewrites (`distributed/fleet/static_meta.py`;
reference `fleet/meta_optimizers/{amp,recompute,gradient_merge,fp16_allreduce}_optimizer.py`):
each rewrite's ops are in the program, and training through it matches the plain run — single
process and 2-rank gloo data parallel; amp's loss scaling skips and rescales on inf/nan."""
import re

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.distributed import fleet

from dist_utils import run_distributed

B = 8


def _program(seed=0, depth=4):
    torch.manual_seed(seed)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [None, 8], "float32")
        y = static.data("y", [None, 1], "float32")
        h, hs = x, []
        for _ in range(depth - 1):
            h = static.nn.fc(h, 16, activation="relu")
            hs.append(h)
        pred = static.nn.fc(h, 1)
        loss = paddle.mean((pred - y) ** 2)
    return main, startup, loss, hs


def _feeds(n, bsz=B, seed=1):
    r = np.random.RandomState(seed)
    return [(r.randn(bsz, 8).astype("float32"), r.randn(bsz, 1).astype("float32")) for _ in range(n)]


def _train(flags=None, feeds=None, rank=0, world=1, opt="sgd", checkpoints=False, fleet_on=True,
           inject=None):
    """Build + run; returns (losses, params, op types)."""
    paddle.enable_static()
    try:
        main, startup, loss, hs = _program()
        with static.program_guard(main, startup):
            o = (paddle.optimizer.SGD(learning_rate=0.1) if opt == "sgd"
                 else paddle.optimizer.Adam(learning_rate=0.01))
            if fleet_on:
                st = fleet.DistributedStrategy()
                for k, v in (flags or {}).items():
                    setattr(st, k, v)
                if checkpoints:
                    st.recompute_configs = {"checkpoints": [hs[0], hs[2]]}
                fleet.init(is_collective=True, strategy=st)
                o = fleet.distributed_optimizer(o)
            o.minimize(loss)
        types = [op.type for op in main.global_block().ops]
        for blk in main.blocks[1:]:
            types += [op.type for op in blk.ops]
        exe = static.Executor("cpu")
        scope = static.Scope()
        losses = []
        with static.scope_guard(scope):
            for i, (X, Y) in enumerate(feeds):
                if world > 1:
                    X, Y = np.split(X, world)[rank], np.split(Y, world)[rank]
                if inject is not None and i == inject:
                    X = X.copy()
                    X[0, 0] = np.inf
                out, = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])
                losses.append(float(np.asarray(out).reshape(-1)[0]))
            # program order (unique-name counters differ between programs)
            params = [scope.get(n).detach().clone() for n in main.params
                      if re.fullmatch(r"linear_\d+\.[wb]_\d+", n)]
            extra = {n: scope.get(n).detach().clone() for n in ("loss_scaling_0",) if scope.get(n) is not None}
        return losses, params, types, extra
    finally:
        paddle.disable_static()


def _close_params(a, b, tol=1e-5):
    assert len(a) == len(b) == 8
    for x, y in zip(a, b):
        torch.testing.assert_close(torch.as_tensor(x), y, rtol=tol, atol=tol)


# ----------------------------------------------------------------------------- gradient merge
def test_gradient_merge_equals_large_batch():
    micro = _feeds(4)
    big = [(np.concatenate([micro[i][0], micro[i + 1][0]]), np.concatenate([micro[i][1], micro[i + 1][1]]))
           for i in (0, 2)]
    ref_l, ref_p, _, _ = _train(feeds=big, fleet_on=False)
    l, p, types, _ = _train({"gradient_merge": True, "gradient_merge_configs": {"k_steps": 2, "avg": True}}, micro)
    assert "conditional_block" in types and types.count("sgd") == 8
    _close_params(p, ref_p)


# ----------------------------------------------------------------------------- recompute
@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_recompute_matches_plain_training(opt):
    f = _feeds(3)
    ref_l, ref_p, _, _ = _train(feeds=f, fleet_on=False, opt=opt)
    l, p, types, _ = _train({"recompute": True}, f, opt=opt, checkpoints=True)
    np.testing.assert_allclose(l, ref_l, rtol=1e-6, atol=1e-7)
    _close_params(p, ref_p)


def test_recompute_program_reemits_segment():
    paddle.enable_static()
    try:
        main, startup, loss, hs = _program()
        with static.program_guard(main, startup):
            st = fleet.DistributedStrategy()
            st.recompute = True
            st.recompute_configs = {"checkpoints": [hs[0], hs[2]]}
            fleet.init(is_collective=True, strategy=st)
            fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.1)).minimize(loss)
        ops = main.global_block().ops
        copies = [op for op in ops if op.attrs.get("_recompute_copy")]
        origs = [op for op in ops if op.attrs.get("_recompute_fwd")]
        assert copies and len(copies) == len(origs)
        names = [n for op in copies for n in op.output_names()]
        assert all(n.endswith("@RECOMPUTE") for n in names)
        first_grad = min(i for i, op in enumerate(ops) if op.type.endswith("_grad"))
        assert min(ops.index(c) for c in copies) > first_grad  # emitted inside the backward pass
    finally:
        paddle.disable_static()


# ----------------------------------------------------------------------------- amp
def test_amp_bf16_casts_and_trains_close_to_fp32():
    f = _feeds(3)
    ref_l, ref_p, _, _ = _train(feeds=f, fleet_on=False)
    l, p, types, _ = _train({"amp": True, "amp_configs": {"use_bf16": True}}, f)
    assert types.count("cast") >= 4
    np.testing.assert_allclose(l, ref_l, rtol=3e-2, atol=3e-2)
    for a, b in zip(p, ref_p):
        assert a.dtype == torch.float32
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2)


def test_amp_fp16_loss_scaling_ops_and_inf_skip():
    f = _feeds(4)
    cfg = {"use_bf16": False, "init_loss_scaling": 1024.0, "decr_every_n_nan_or_inf": 1,
           "incr_every_n_steps": 1000}
    l, p, types, extra = _train({"amp": True, "amp_configs": cfg}, f)
    assert "check_finite_and_unscale" in types and "update_loss_scaling" in types
    ref_l, ref_p, _, _ = _train(feeds=f, fleet_on=False)
    np.testing.assert_allclose(l, ref_l, rtol=3e-2, atol=3e-2)
    # an inf in the last step's input: that update is skipped and the scale halves
    l3, p3, _, e3 = _train({"amp": True, "amp_configs": cfg}, f[:3])
    li, pi, _, ei = _train({"amp": True, "amp_configs": cfg}, f, inject=3)
    _close_params(pi, p3)
    assert float(ei["loss_scaling_0"]) == 512.0 and float(e3["loss_scaling_0"]) == 1024.0


def test_amp_fp16_with_gradient_merge_unscales_merged_grads_once_per_k():
    """AMP + gradient merge: check_finite_and_unscale / update_loss_scaling run inside the
    every-k block on the merged gradients. An inf in the FIRST micro-step of a window skips that
    window's update (merged grads zeroed) and halves the scale once; the next window trains as if
    the first never happened."""
    f = _feeds(4)
    cfg = {"use_bf16": False, "init_loss_scaling": 1024.0, "decr_every_n_nan_or_inf": 1,
           "incr_every_n_steps": 1000}
    flags = {"amp": True, "amp_configs": cfg, "gradient_merge": True,
             "gradient_merge_configs": {"k_steps": 2, "avg": True}}
    l, p, types, extra = _train(flags, f)
    assert types.count("check_finite_and_unscale") == 1 and "conditional_block" in types
    assert float(extra["loss_scaling_0"]) == 1024.0
    li, pi, _, ei = _train(flags, f, inject=0)
    assert float(ei["loss_scaling_0"]) == 512.0  # one decrement for the whole window
    for t in pi:
        assert torch.isfinite(torch.as_tensor(t)).all()
    l2, p2, _, _ = _train(flags, f[2:])
    _close_params(pi, p2, tol=2e-3)


# ----------------------------------------------------------------------------- 2-rank gloo
def _dp_worker(rank, world, flags, checkpoints):
    feeds = _feeds(4, 2 * B)
    return _train(flags, feeds, rank, world, checkpoints=checkpoints)[:2]


@pytest.mark.parametrize("case", ["gm", "recompute", "fp16_allreduce", "amp_bf16"])
def test_two_rank_data_parallel_matches_single(case):
    flags = {"gm": {"gradient_merge": True, "gradient_merge_configs": {"k_steps": 2, "avg": True}},
             "recompute": {"recompute": True},
             "fp16_allreduce": {"fp16_allreduce": True},
             "amp_bf16": {"amp": True, "amp_configs": {"use_bf16": True}}}[case]
    res = run_distributed(_dp_worker, 2, flags, case == "recompute")
    micro = _feeds(4, 2 * B)
    if case == "gm":  # single process: one update per two full batches
        feeds = [(np.concatenate([micro[i][0], micro[i + 1][0]]), np.concatenate([micro[i][1], micro[i + 1][1]]))
                 for i in (0, 2)]
        _, ref_p, _, _ = _train(feeds=feeds, fleet_on=False)
    else:
        _, ref_p, _, _ = _train(feeds=micro, fleet_on=False)
    tol = {"gm": 1e-5, "recompute": 1e-5, "fp16_allreduce": 2e-3, "amp_bf16": 6e-2}[case]
    for r in range(2):
        _close_params(res[r][1], ref_p, tol)

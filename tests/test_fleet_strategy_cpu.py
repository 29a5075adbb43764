"""Every DistributedStrategy switch is honoured or rejected (reference `fleet/meta_optimizers/`:
amp / recompute / gradient_merge / lamb / lars / asp meta-optimizers, `raw_program_optimizer.py`
for static data parallelism): one test per flag showing its effect, or its error."""
import copy

import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.distributed import fleet

from dist_utils import run_distributed


def _init(**flags):
    st = fleet.DistributedStrategy()
    for k, v in flags.items():
        setattr(st, k, v)
    fleet.init(is_collective=True, strategy=st)
    return st


def _mlp(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(paddle.nn.Linear(8, 16), torch.nn.ReLU(), paddle.nn.Linear(16, 1))


def _batches(n=4, B=8, seed=1):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(B, 8, generator=g), torch.randn(B, 1, generator=g)) for _ in range(n)]


def test_unknown_field_and_config_key_raise():
    st = fleet.DistributedStrategy()
    with pytest.raises(AttributeError):
        st.not_a_field = True
    with pytest.raises(ValueError):
        st.sharding_configs = {"stage": 3, "bogus": 1}
    with pytest.raises(ValueError):
        st.hybrid_configs = {"dp_degree": 1, "xp_degree": 2}
    st.sharding_configs = {"stage": 3}  # merged into the defaults, like the reference
    assert st.sharding_configs["stage"] == 3 and "segment_broadcast_MB" in st.sharding_configs


@pytest.mark.parametrize("flag", ["a_sync",
                                  "heter_ccl_mode", "auto", "semi_auto", "qat"])
def test_unsupported_switches_raise(flag):
    st = fleet.DistributedStrategy()
    setattr(st, flag, True)
    with pytest.raises(NotImplementedError, match=flag):
        fleet.init(is_collective=True, strategy=st)


def test_gradient_merge_updates_every_k_steps_with_averaged_grads():
    _init(gradient_merge=True, gradient_merge_configs={"k_steps": 2, "avg": True})
    m = _mlp()
    ref = copy.deepcopy(m)
    model = fleet.distributed_model(m)
    opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.5, parameters=m.parameters()))
    (x1, y1), (x2, y2) = _batches(2)
    p0 = [p.detach().clone() for p in m.parameters()]
    for i, (x, y) in enumerate(((x1, y1), (x2, y2))):
        loss = torch.mean((model(x) - y) ** 2)
        loss.backward()
        opt.step()
        opt.clear_grad()
        if i == 0:  # no update yet, gradients kept
            for a, b in zip(m.parameters(), p0):
                assert torch.equal(a.detach(), b)
    # reference: one SGD step on the mean of the two batches' gradients
    l1 = torch.mean((ref(x1) - y1) ** 2)
    l2 = torch.mean((ref(x2) - y2) ** 2)
    ((l1 + l2) / 2).backward()
    with torch.no_grad():
        for p in ref.parameters():
            p -= 0.5 * p.grad
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)


def test_lamb_replaces_adam():
    _init(lamb=True, lamb_configs={"lamb_weight_decay": 0.02})
    m = _mlp()
    fleet.distributed_model(m)
    opt = fleet.distributed_optimizer(paddle.optimizer.Adam(learning_rate=0.01, parameters=m.parameters()))
    assert isinstance(opt._inner, paddle.optimizer.Lamb) and opt._inner._wd == 0.02
    losses = []
    for x, y in _batches(8, seed=2) * 3:
        loss = torch.mean((m(x) - y) ** 2)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0]
    with pytest.raises(TypeError):
        fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters()))


def test_lars_replaces_momentum_with_the_lars_rule():
    _init(lars=True, lars_configs={"lars_coeff": 0.01, "lars_weight_decay": 0.001})
    lin = paddle.nn.Linear(4, 3)
    fleet.distributed_model(lin)
    opt = fleet.distributed_optimizer(paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9,
                                                                parameters=lin.parameters()))
    assert isinstance(opt._inner, paddle.optimizer.LarsMomentum)
    w0 = lin.weight.detach().clone()
    x = torch.randn(5, 4)
    lin(x).sum().backward()
    g = lin.weight.grad.detach().clone()
    opt.step()
    wn, gn = w0.norm(), g.norm()
    local = 0.1 * 0.01 * wn / (gn + 0.001 * wn)
    torch.testing.assert_close(lin.weight.detach(), w0 - local * (g + 0.001 * w0), rtol=1e-5, atol=1e-7)


def test_amp_runs_forward_in_bf16():
    _init(amp=True, amp_configs={"use_bf16": True})
    lin = paddle.nn.Linear(8, 8)
    model = fleet.distributed_model(lin)
    out = model(torch.randn(2, 8))
    assert out.dtype == torch.bfloat16
    assert lin.weight.dtype == torch.float32  # O1: weights stay fp32


def test_amp_o2_casts_weights_but_not_norms():
    _init(amp=True, amp_configs={"use_pure_fp16": True, "use_bf16": True})
    m = torch.nn.Sequential(paddle.nn.Linear(8, 8), paddle.nn.LayerNorm(8))
    fleet.distributed_model(m)
    assert m[0].weight.dtype == torch.bfloat16 and m[1].weight.dtype == torch.float32


def test_recompute_switches_model_recompute_and_matches_grads():
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    _init(recompute=True)
    cfg = gpt_config("gpt3-tiny", dtype="float32", num_layers=2, hidden_size=32, num_heads=2,
                     vocab_size=64, max_position_embeddings=32, hidden_dropout_prob=0.0)
    gpt = GPTForPretraining(cfg)
    fleet.distributed_model(gpt)
    assert gpt.cfg.recompute
    # generic model: every LayerList / Sequential element re-runs in backward, same gradients
    _init(recompute=True)
    m = _mlp()
    ref = copy.deepcopy(m)
    fleet.distributed_model(m)
    assert all(getattr(c, "_fleet_recompute", False) for c in m.children())
    x = torch.randn(4, 8, requires_grad=True)
    m(x).square().sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    ref(xr).square().sum().backward()
    torch.testing.assert_close(x.grad, xr.grad)
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a.grad, b.grad)


def test_sync_batch_norm_converts_layers():
    _init(sync_batch_norm=True)
    m = torch.nn.Sequential(paddle.nn.Conv2D(3, 4, 3), paddle.nn.BatchNorm2D(4))
    fleet.distributed_model(m)
    assert type(m[1]).__name__ == "SyncBatchNorm"


def test_asp_keeps_2_4_sparsity_through_updates():
    from paddle_infer_amd.incubate import asp
    _init(asp=True)
    lin = paddle.nn.Linear(16, 8)
    asp.prune_model(lin)
    fleet.distributed_model(lin)
    opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.1, parameters=lin.parameters()))
    lin(torch.randn(4, 16)).sum().backward()
    opt.step()
    w = lin.weight.detach().t().reshape(-1, 4)  # [in, out]: groups of 4 along the reduction dim
    assert int((w != 0).sum(-1).max()) <= 2


# ------------------------------------------------------------------------ static-graph fleet
def _static_program(seed=0):
    torch.manual_seed(seed)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data("x", [None, 8], "float32")
        y = static.data("y", [None, 1], "float32")
        h = static.nn.fc(x, 16, activation="relu")
        pred = static.nn.fc(h, 1)
        loss = paddle.mean((pred - y) ** 2)
    return main, startup, loss


def _feeds(n=3, B=8, seed=1):
    r = np.random.RandomState(seed)
    return [(r.randn(B, 8).astype("float32"), r.randn(B, 1).astype("float32")) for _ in range(n)]


def _static_train(rank=0, world=1, use_fleet=False):
    paddle.enable_static()
    try:
        main, startup, loss = _static_program()
        with static.program_guard(main, startup):
            opt = paddle.optimizer.SGD(learning_rate=0.1)
            if use_fleet:
                _init()
                opt = fleet.distributed_optimizer(opt)
            opt.minimize(loss)
        types = [op.type for op in main.global_block().ops]
        exe = static.Executor("cpu")
        scope = static.Scope()
        with static.scope_guard(scope):
            for X, Y in _feeds():
                xs, ys = np.split(X, world)[rank], np.split(Y, world)[rank]
                exe.run(main, feed={"x": xs, "y": ys}, fetch_list=[loss])
            params = [scope.get(n).detach().clone() for n in main.params if not n.startswith("learning_rate")]
        return params, types
    finally:
        paddle.disable_static()


def _static_fleet_worker(rank, world):
    return _static_train(rank, world, True)


def test_static_fleet_minimize_inserts_allreduce_and_matches_single():
    ref, _ = _static_train()
    res = run_distributed(_static_fleet_worker, 2)
    for r in range(2):
        params, types = res[r]
        assert types.count("c_allreduce_sum") == 4 and "scale" in types
        first_opt = min(i for i, t in enumerate(types) if t in ("sgd", "optimize"))
        assert max(i for i, t in enumerate(types) if t == "c_allreduce_sum") < first_opt
        for a, b in zip(params, ref):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)

"""paddle.distributed API on CPU gloo (world 2): collectives, DataParallel, 1F1B pipeline,
group-sharded stage 3, fleet hybrid optimizer, recompute and the launcher watchdog."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

from dist_utils import run_distributed


def _collectives(rank, world):
    import paddle_infer_amd.distributed as pd
    x = torch.tensor([float(rank + 1)] * 4)
    pd.all_reduce(x)
    out = []
    pd.all_gather(out, torch.tensor([rank]))
    a2a = []
    pd.alltoall([torch.tensor([rank * 10 + i]) for i in range(world)], a2a)
    rs = torch.empty(2)
    pd.reduce_scatter(rs, [torch.ones(2) * (rank + 1), torch.ones(2) * (rank + 1)])
    objs = []
    pd.all_gather_object(objs, {"r": rank})
    return x.tolist(), [t.item() for t in out], [t.item() for t in a2a], rs.tolist(), objs


def test_collectives():
    res = run_distributed(_collectives, 2)
    for r in range(2):
        x, ag, a2a, rs, objs = res[r]
        assert x == [3.0] * 4 and ag == [0, 1]
        assert a2a == [0 * 10 + r, 1 * 10 + r]
        assert rs == [3.0, 3.0] and objs == [{"r": 0}, {"r": 1}]


def _mlp():
    import paddle_infer_amd as paddle
    torch.manual_seed(0)
    return paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 16),
                                paddle.nn.ReLU(), paddle.nn.Linear(16, 4))


def _data():
    g = torch.Generator().manual_seed(3)
    return torch.randn(8, 8, generator=g), torch.randn(8, 4, generator=g)


def _single_sgd(steps=2):
    import paddle_infer_amd as paddle
    m = _mlp()
    o = paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters())
    x, y = _data()
    for _ in range(steps):
        loss = ((m(x) - y) ** 2).mean()
        loss.backward()
        o.step()
        o.clear_grad()
    return {k: v.clone() for k, v in m.state_dict().items()}


def _dp_worker(rank, world):
    import paddle_infer_amd as paddle
    import paddle_infer_amd.distributed as pd
    m = pd.DataParallel(_mlp(), comm_buffer_size=0.0005)
    o = paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters())
    x, y = _data()
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    for _ in range(2):
        loss = ((m(xs) - ys) ** 2).mean()
        loss.backward()
        o.step()
        o.clear_grad()
    return {k: v.clone() for k, v in m.state_dict().items()}


def test_data_parallel_generic_model():
    ref = _single_sgd()
    res = run_distributed(_dp_worker, 2)
    for r in range(2):
        for k in ref:
            torch.testing.assert_close(res[r][k], ref[k], rtol=1e-5, atol=1e-6)


def _pp_worker(rank, world):
    import paddle_infer_amd as paddle
    from paddle_infer_amd.distributed import fleet
    from paddle_infer_amd.distributed.fleet import LayerDesc, PipelineLayer
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {"dp_degree": 1, "mp_degree": 1, "pp_degree": 2,
                         "pp_configs": {"accumulate_steps": 4, "micro_batch_size": 2}}
    fleet.init(is_collective=True, strategy=st)
    torch.manual_seed(0)
    full = _mlp()
    descs = list(full.children())
    loss_fn = lambda out, y: ((out - y) ** 2).mean()  # noqa: E731
    pl = PipelineLayer(descs, num_stages=2, loss_fn=loss_fn)
    model = fleet.distributed_model(pl)
    opt = paddle.optimizer.SGD(learning_rate=0.1, parameters=pl.parameters())
    x, y = _data()
    losses = []
    for _ in range(2):
        losses.append(float(model.train_batch([x, y], opt)))
    return {"stage": pl.stage_id, "sd": {k: v.clone() for k, v in full.state_dict().items()}, "losses": losses}


def test_pipeline_1f1b_matches_single():
    import paddle_infer_amd as paddle
    m = _mlp()
    o = paddle.optimizer.SGD(learning_rate=0.1, parameters=m.parameters())
    x, y = _data()
    ref_losses = []
    for _ in range(2):
        tot = 0.0
        for xs, ys in zip(x.chunk(4), y.chunk(4)):
            loss = ((m(xs) - ys) ** 2).mean() / 4
            loss.backward()
            tot += loss.item()
        ref_losses.append(tot)
        o.step()
        o.clear_grad()
    ref = m.state_dict()
    res = run_distributed(_pp_worker, 2)
    for r in range(2):
        assert res[r]["losses"] == pytest.approx(ref_losses, rel=1e-5)
    # stage 0 owns layers 0..2, stage 1 owns 3..4 (uniform split of 5 descs)
    s0 = res[0]["sd"] if res[0]["stage"] == 0 else res[1]["sd"]
    s1 = res[1]["sd"] if res[1]["stage"] == 1 else res[0]["sd"]
    torch.testing.assert_close(s0["0.weight"], ref["0.weight"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(s1["4.weight"], ref["4.weight"], rtol=1e-5, atol=1e-6)


def _stage3_worker(rank, world):
    import paddle_infer_amd as paddle
    import paddle_infer_amd.distributed as pd
    m = _mlp()
    o = paddle.optimizer.AdamW(learning_rate=0.01, parameters=m.parameters(), weight_decay=0.0)
    m3, o3, _ = pd.group_sharded_parallel(m, o, "p_g_os")
    x, y = _data()
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    for _ in range(2):
        loss = ((m3(xs) - ys) ** 2).mean()
        loss.backward()
        o3.step()
        o3.clear_grad()
    return {k: v.clone() for k, v in m3.state_dict().items()}


def test_group_sharded_stage3_matches_single():
    import paddle_infer_amd as paddle
    m = _mlp()
    o = paddle.optimizer.AdamW(learning_rate=0.01, parameters=m.parameters(), weight_decay=0.0)
    x, y = _data()
    for _ in range(2):
        loss = ((m(x) - y) ** 2).mean()
        loss.backward()
        o.step()
        o.clear_grad()
    ref = m.state_dict()
    res = run_distributed(_stage3_worker, 2)
    for r in range(2):
        for k in ref:
            torch.testing.assert_close(res[r][k], ref[k], rtol=1e-4, atol=1e-5)


def test_recompute_matches_plain():
    from paddle_infer_amd.distributed.fleet import recompute
    import paddle_infer_amd.nn.functional as F
    torch.manual_seed(0)
    lin = torch.nn.Linear(8, 8)
    x = torch.randn(4, 8, requires_grad=True)

    def f(t):
        return F.dropout(torch.tanh(lin(t)), 0.5, training=True)
    torch.manual_seed(5)
    y1 = f(x).sum()
    y1.backward()
    g1 = [x.grad.clone(), lin.weight.grad.clone()]
    x.grad, lin.weight.grad = None, None
    torch.manual_seed(5)
    y2 = recompute(f, x).sum()
    y2.backward()
    g2 = [x.grad, lin.weight.grad]
    assert y1.item() == pytest.approx(y2.item())
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b)


def test_launch_watchdog_kills_job_on_failure(tmp_path):
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)
    """))
    import time as _t
    t0 = _t.time()
    r = subprocess.run([sys.executable, "-m", "paddle_infer_amd.distributed.launch",
                        "--nproc_per_node", "2", "--log_dir", str(tmp_path / "log"), str(script)],
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
    assert _t.time() - t0 < 30
    assert (tmp_path / "log" / "workerlog.0").exists()


def _ckpt_worker(rank, world, path, phase):
    import torch
    import torch.distributed as dist
    from paddle_infer_amd.distributed import checkpoint as ck
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    from paddle_infer_amd.parallel.flat_engine import FlatTrainer
    torch.manual_seed(0)
    cfg = gpt_config("gpt3-tiny", dtype="float32", hidden_dropout_prob=0.0, num_layers=1)
    m = GPTForPretraining(cfg)
    tr = FlatTrainer(m, lr=1e-2, dp_group=dist.group.WORLD, sharding_stage=1, bucket_mb=0.05)
    if phase == "save":
        ids = torch.randint(0, cfg.vocab_size, (2, 17), generator=torch.Generator().manual_seed(rank))
        tr.zero_grad()
        m(ids[:, :-1], labels=ids[:, 1:]).backward()
        tr.step()
        tr.wait_params()
        ck.save_state_dict(ck.flat_trainer_state(tr, m), path)
        full = {g.name: g.master.clone() for g in tr.groups}
        return {"step": tr.step_count, "params": {k: v.clone() for k, v in m.state_dict().items()},
                "shards": {k: v.numpy() for k, v in full.items()}}
    st = ck.flat_trainer_state(tr, m)
    extra = ck.load_state_dict(st, path)
    return {"step": extra.get("opt.step"), "params": {k: v.clone() for k, v in m.state_dict().items()},
            "shards": {g.name: g.master.numpy().copy() for g in tr.groups}}


def test_distributed_checkpoint_reshards(tmp_path):
    """Save with world 2 (ZeRO-1 shards), load with world 1 and world 2: params identical, and the
    world-1 master equals the concatenation (per bucket) of the world-2 shards."""
    path = str(tmp_path / "ckpt")
    saved = run_distributed(_ckpt_worker, 2, path, "save")
    loaded2 = run_distributed(_ckpt_worker, 2, path, "load")
    loaded1 = _ckpt_worker(0, 1, path, "load")
    for r in range(2):
        for k, v in saved[0]["params"].items():
            torch.testing.assert_close(loaded2[r]["params"][k], v)
        for name, arr in saved[r]["shards"].items():
            np.testing.assert_allclose(loaded2[r]["shards"][name], arr)
    for k, v in saved[0]["params"].items():
        torch.testing.assert_close(loaded1["params"][k], v)
    assert loaded1["step"] == 1


def _tp_ckpt_worker(rank, world, path, phase):
    import torch.distributed as dist  # noqa: F401
    from paddle_infer_amd.distributed import checkpoint as ck
    g = torch.arange(6 * 8 * 4, dtype=torch.float32).reshape(6, 8, 4)
    if phase == "save":  # TP=2: column split on axis 1, row split on axis 0
        col = g.chunk(world, dim=1)[rank]
        row = g.chunk(world, dim=0)[rank]
        ck.save_state_dict({"col": ck.axis_shard(col, g.shape, 1, rank, world),
                            "row": ck.axis_shard(row, g.shape, 0, rank, world), "step": 5}, path)
        return {}
    return {}


def test_checkpoint_tensor_parallel_reshard(tmp_path):
    """Save TP=2 column/row shards from 2 ranks; load as full tensors (world 1) and as TP=4 /
    other-axis shards."""
    from paddle_infer_amd.distributed import checkpoint as ck
    path = str(tmp_path / "tp")
    run_distributed(_tp_ckpt_worker, 2, path, "save")
    g = torch.arange(6 * 8 * 4, dtype=torch.float32).reshape(6, 8, 4)
    full_col, full_row = torch.zeros_like(g), torch.zeros_like(g)
    extra = ck.load_state_dict({"col": full_col, "row": full_row}, path)
    assert extra["step"] == 5
    torch.testing.assert_close(full_col, g)
    torch.testing.assert_close(full_row, g)
    for r in range(4):  # TP=4 along axis 1 from the axis-1 TP=2 checkpoint, axis 2 from axis 0
        a = torch.zeros(6, 2, 4)
        b = torch.zeros(6, 8, 1)
        sa, sb = ck.axis_shard(a, g.shape, 1, r, 4), ck.axis_shard(b, g.shape, 2, r, 4)
        ck.load_state_dict({"col": sa, "row": sb}, path)
        torch.testing.assert_close(sa.local.view(6, 2, 4), g.chunk(4, dim=1)[r])
        torch.testing.assert_close(sb.local.view(6, 8, 1), g.chunk(4, dim=2)[r])


def _auto_parallel_worker(rank, world):
    import torch
    import paddle_infer_amd.distributed as pd
    from paddle_infer_amd.distributed.communication import stream
    torch.manual_seed(0)
    full_w = torch.randn(8, 6)
    x = torch.randn(3, 8)
    mesh = pd.ProcessMesh([0, 1], ["mp"])
    w = pd.shard_tensor(full_w, mesh, [None, "mp"])  # column split
    local = w.to_local()
    y = torch.nn.functional.linear(x, full_w.t()[rank * 3:(rank + 1) * 3])
    back = pd.reshard(w, mesh, [None, None]).to_local()
    t = torch.full((2,), float(rank + 1))
    stream.all_reduce(t, use_calc_stream=True)
    g = torch.zeros(4)
    stream.all_gather(g, torch.full((2,), float(rank)))
    return {"local": local, "ref_cols": full_w[:, rank * 3:(rank + 1) * 3], "y": y,
            "back": back, "full": full_w, "ar": t, "ag": g}


def test_auto_parallel_shard_tensor_and_stream_collectives():
    res = run_distributed(_auto_parallel_worker, 2)
    for r in res.values():
        assert torch.allclose(r["local"], r["ref_cols"])
        assert torch.allclose(r["back"], r["full"])
        assert torch.equal(r["ar"], torch.full((2,), 3.0))
        assert torch.equal(r["ag"], torch.tensor([0.0, 0.0, 1.0, 1.0]))


def test_auto_parallel_engine_single_process():
    import paddle_infer_amd as paddle
    from paddle_infer_amd.distributed.auto_parallel import Engine, Strategy
    torch.manual_seed(0)
    model = paddle.nn.Linear(4, 1)
    opt = paddle.optimizer.SGD(0.1, parameters=model.parameters())
    X = torch.randn(64, 4)
    Y = X @ torch.tensor([[1.0], [-2.0], [0.5], [3.0]])
    data = paddle.io.TensorDataset([X, Y])
    st = Strategy({"gradient_merge": {"enable": True, "k_steps": 2}})
    eng = Engine(model, paddle.nn.MSELoss(), opt, strategy=st)
    hist = eng.fit(data, batch_size=8, epochs=20)
    assert hist["loss"][-1] < hist["loss"][0] * 0.1
    assert eng.evaluate(data, batch_size=16)["loss"] < hist["loss"][0] * 0.1

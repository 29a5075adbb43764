"""Static auto-parallel completion + partition (distributed/auto_parallel/partitioner.py;
reference `auto_parallel/completion.py`, `partitioner.py`, `reshard.py`): a serial static program
annotated with ``shard_tensor`` is partitioned per rank over 2 gloo processes (and a 2x2 mesh over
4), and every rank's partitioned program reproduces the serial outputs."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.distributed import auto_parallel as auto

from dist_utils import run_distributed


def _build(mesh_shape, specs, seed=0):
    """Embedding -> fused QKV linear -> heads (reshape/transpose) -> attention matmuls + softmax ->
    out-proj -> residual + LayerNorm -> FFN (gelu) -> mean over hidden."""
    import paddle_infer_amd.nn as nn
    import paddle_infer_amd.nn.functional as F
    torch.manual_seed(seed)
    main, startup = static.Program(), static.Program()
    mesh = auto.ProcessMesh(np.arange(int(np.prod(mesh_shape))).reshape(mesh_shape).tolist(),
                            ["dp", "mp"][-len(mesh_shape):] if len(mesh_shape) == 1 else ["dp", "mp"])
    with static.program_guard(main, startup):
        ids = static.data("ids", [4, 6], "int64")
        emb = nn.Embedding(32, 16)
        q_l, k_l, v_l = nn.Linear(16, 16), nn.Linear(16, 16), nn.Linear(16, 16)
        o_l, f1, f2 = nn.Linear(16, 16), nn.Linear(16, 32), nn.Linear(32, 16)
        ln = nn.LayerNorm(16)
        for t, key in ((emb.weight, "emb"), (q_l.weight, "col"), (k_l.weight, "col"), (v_l.weight, "col"),
                       (q_l.bias, "colb"), (k_l.bias, "colb"), (v_l.bias, "colb"), (o_l.weight, "row"),
                       (f1.weight, "col"), (f1.bias, "colb"), (f2.weight, "row")):
            if specs.get(key) is not None:
                auto.shard_tensor(t, mesh, specs[key])
        if specs.get("ids") is not None:
            auto.shard_tensor(ids, mesh, specs["ids"])
        h = emb(ids)

        def heads(t):
            return paddle.reshape(t, [4, 6, 4, 4]).transpose([0, 2, 1, 3])
        q, k, v = heads(q_l(h)), heads(k_l(h)), heads(v_l(h))
        s = paddle.matmul(q, k, transpose_y=True) * 0.5
        p = F.softmax(s, axis=-1)
        o = paddle.matmul(p, v).transpose([0, 2, 1, 3])
        o = paddle.reshape(o, [4, 6, 16])
        y = ln(o_l(o) + h)
        z = f2(F.gelu(f1(y))) + y
        out = paddle.mean(z, axis=-1)
    return main, mesh, out, z


def _ids():
    return np.random.RandomState(3).randint(0, 32, size=(4, 6)).astype("int64")


def _serial(mesh_shape, specs):
    paddle.enable_static()
    try:
        main, mesh, out, z = _build(mesh_shape, specs)
        exe = static.Executor("cpu")
        with static.scope_guard(static.Scope()):
            return exe.run(main, feed={"ids": _ids()}, fetch_list=[out, z])
    finally:
        paddle.disable_static()


MP = {"emb": ["mp", None], "col": [None, "mp"], "colb": ["mp"], "row": ["mp", None]}


def _worker(rank, world, mesh_shape, specs):
    paddle.enable_static()
    try:
        main, mesh, out, z = _build(mesh_shape, specs)
        c = auto.complete(main, mesh)
        local = auto.Partitioner(c).partition(rank, fetch_list=[out, z])
        kinds = [op.type for op in local.global_block().ops]
        shapes = {n: tuple(t.shape) for n, t in local.params.items()}
        exe = static.Executor("cpu")
        with static.scope_guard(static.Scope()):
            res = exe.run(local, feed={"ids": _ids()}, fetch_list=[out, z])
        return res, kinds, shapes
    finally:
        paddle.disable_static()


@pytest.mark.parametrize("mesh_shape,specs", [((2,), MP), ((2, 2), dict(MP, ids=["dp", None]))])
def test_partitioned_programs_match_serial(mesh_shape, specs):
    world = int(np.prod(mesh_shape))
    ref = _serial(mesh_shape, {})
    res = run_distributed(_worker, world, mesh_shape, specs)
    for r in range(world):
        (o, z), kinds, shapes = res[r]
        np.testing.assert_allclose(o, ref[0], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(z, ref[1], rtol=1e-4, atol=1e-5)
        # column-parallel weights hold half the output features, row-parallel half the inputs
        assert (16, 8) in shapes.values() and (8, 16) in shapes.values() and (16, 16) in shapes.values()
        assert (32, 16) not in shapes.values()  # FFN1 column split -> (16, 16); emb vocab split -> (16, 16)
        # Megatron pattern: one all-reduce per row-parallel linear + the vocab-parallel embedding,
        # no all-gather inside the attention block (heads stay split through reshape/transpose)
        assert kinds.count("c_allreduce_sum") == 0  # row-parallel linears with bias reduce inside
        # heads stay split through reshape / transpose / both attention matmuls / softmax: no
        # all-gather inside the layer; with a dp-split batch only the two fetched outputs gather
        assert kinds.count("c_allgather") == (0 if len(mesh_shape) == 1 else 2), kinds


def test_completion_propagates_head_split_through_reshape_transpose():
    paddle.enable_static()
    try:
        main, mesh, out, z = _build((2,), MP)
        c = auto.complete(main, mesh)
    finally:
        paddle.disable_static()
    maps = {tuple(a.dims_mapping) for a in c.attrs.values()}
    # q/k/v heads [4, 4(h), 6, 4] split on the head dim after reshape + transpose
    assert (-1, 0, -1, -1) in maps
    # no reshard was needed for the attention matmuls (their inputs already agree)
    mm = [p for p in c.plans if p["op"].type == "matmul_v2"]
    assert mm and all(not p["req"] for p in mm)


def _train_losses(mesh_shape, specs, rank=None, steps=3):
    paddle.enable_static()
    try:
        main, mesh, out, z = _build(mesh_shape, specs)
        with static.program_guard(main, static.Program()):  # the loss belongs to the serial program
            loss = paddle.mean(out * out)
        prog = main
        if rank is not None:
            prog = auto.partition(main, mesh, rank)
        with static.program_guard(prog, static.Program()):
            loss = prog.global_block().vars[loss.var_name]
            paddle.optimizer.SGD(learning_rate=0.5).minimize(loss)
        exe = static.Executor("cpu")
        losses = []
        with static.scope_guard(static.Scope()):
            for _ in range(steps):
                (lv,) = exe.run(prog, feed={"ids": _ids()}, fetch_list=[loss])
                losses.append(float(lv))
        return losses
    finally:
        paddle.disable_static()


def _train_worker(rank, world, mesh_shape, specs):
    return _train_losses(mesh_shape, specs, rank)


@pytest.mark.parametrize("mesh_shape,specs", [((2,), MP), ((2, 2), dict(MP, ids=["dp", None]))])
def test_partitioned_training_matches_serial(mesh_shape, specs):
    """Static training on the partitioned programs (append_backward + SGD after partition): the
    conjugate collectives (all-reduce fwd / identity bwd, c_identity fwd / all-reduce bwd, gather
    fwd / slice bwd, slice fwd / gather bwd) give every rank the serial program's loss curve."""
    ref = _train_losses(mesh_shape, {})
    assert ref[-1] < ref[0]
    res = run_distributed(_train_worker, int(np.prod(mesh_shape)), mesh_shape, specs)
    for r, losses in res.items():
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-6)


def _engine_losses(rank=None, steps=4):
    """Engine.prepare (static trace + completion + partition + backward) then Engine.fit, on an MLP
    whose forward annotates column / row-parallel weights with shard_tensor."""
    import paddle_infer_amd.nn as nn
    import paddle_infer_amd.nn.functional as F
    from paddle_infer_amd.static import InputSpec
    torch.manual_seed(5)
    mesh = auto.ProcessMesh([0, 1], ["mp"])

    class MLP(nn.Layer):
        def __init__(self):
            super().__init__()
            self.l1, self.l2 = nn.Linear(8, 32), nn.Linear(32, 4)

        def forward(self, x):
            if rank is not None:  # the single-process reference runs the unannotated model
                auto.shard_tensor(self.l1.weight, mesh, [None, "mp"])
                auto.shard_tensor(self.l1.bias, mesh, ["mp"])
                auto.shard_tensor(self.l2.weight, mesh, ["mp", None])
            return self.l2(F.gelu(self.l1(x)))

    model = MLP()
    opt = paddle.optimizer.SGD(learning_rate=0.2, parameters=model.parameters())
    eng = auto.Engine(model, paddle.nn.MSELoss(), opt)
    eng.prepare([InputSpec([16, 8], "float32", "x")], [InputSpec([16, 4], "float32", "y")],
                mode="train", process_mesh=mesh if rank is not None else auto.ProcessMesh([0], ["mp"]))
    r = np.random.RandomState(7)
    batch = (torch.as_tensor(r.randn(16, 8).astype("float32")), torch.as_tensor(r.randn(16, 4).astype("float32")))
    data = [batch] * steps  # one batch repeated: the loss must fall step by step
    hist = eng.fit(iter(data), epochs=1)
    kinds = [op.type for op in eng._static["program"].global_block().ops]
    return hist["loss"], kinds


def _engine_worker(rank, world):
    return _engine_losses(rank)


def test_engine_prepare_fit_partitioned_matches_single_process():
    ref, kinds1 = _engine_losses()
    assert "c_allreduce_sum" not in kinds1
    res = run_distributed(_engine_worker, 2)
    for r in range(2):
        losses, kinds = res[r]
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-6)
        assert "c_identity" in kinds  # column-parallel input: all-reduce of its gradient
        assert "sgd" in kinds
    assert ref[-1] < ref[0]


def _gpt_forward(rank=None):
    """The framework's GPT (fused add+LN, packed flash attention, bias-GELU ops) traced to a static
    Program, FFN weights annotated column / row parallel over mp=2."""
    from paddle_infer_amd.models import gpt as G
    paddle.enable_static()
    try:
        torch.manual_seed(0)
        cfg = G.GPTConfig(vocab_size=64, hidden_size=32, num_layers=2, num_heads=4,
                          max_position_embeddings=16, hidden_dropout_prob=0.0, dtype="float32")
        m = G.GPTForPretraining(cfg)
        m.eval()
        mesh = auto.ProcessMesh([0, 1], ["mp"])
        main = static.Program()
        with static.program_guard(main, static.Program()):
            ids = static.data("ids", [2, 8], "int64")
            if rank is not None:
                for L in m.gpt.layers:
                    auto.shard_tensor(L.mlp.fc1.weight, mesh, [None, "mp"])
                    auto.shard_tensor(L.mlp.fc1.bias, mesh, ["mp"])
                    auto.shard_tensor(L.mlp.fc2.weight, mesh, ["mp", None])
            out = m(ids)
            out = out[0] if isinstance(out, (tuple, list)) else out
        prog = main if rank is None else auto.partition(main, mesh, rank, fetch_list=[out])
        feed = {"ids": np.random.RandomState(0).randint(0, 64, (2, 8)).astype("int64")}
        with static.scope_guard(static.Scope()):
            res = static.Executor("cpu").run(prog, feed=feed, fetch_list=[out])[0]
        return res, [op.type for op in prog.global_block().ops]
    finally:
        paddle.disable_static()


def _gpt_worker(rank, world):
    return _gpt_forward(rank)


def test_gpt_program_partitions_megatron_ffn():
    ref, _ = _gpt_forward()
    res = run_distributed(_gpt_worker, 2)
    for r in range(2):
        out, kinds = res[r]
        np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)
        # FFN1 column-parallel -> bias-GELU on the split activations -> FFN2 row-parallel: one
        # all-reduce per layer (bias folded into the next add+LN), no all-gather anywhere
        assert kinds.count("c_allreduce_sum") == 2 and "c_allgather" not in kinds, kinds

"""Multi-stream static executor (`static/streams.py`, native `piamd_stream_plan` in
`csrc/runtime/scheduler.cc`; reference `new_executor/interpreter/stream_analyzer.cc`,
`interpretercore.cc:907`): the stream assignment and minimal cross-stream event waits of a program
with collectives, and 2-rank gloo runs with the collectives issued on the communication stream
(asynchronously) — a tensor-parallel partitioned program and a data-parallel CompiledProgram with
bucketed, backward-overlapped gradient all-reduce — that match the single-process losses."""
import numpy as np
import pytest
import torch

import paddle_infer_amd as paddle
from paddle_infer_amd import static
from paddle_infer_amd.inference.passes import _new
from paddle_infer_amd.static.streams import stream_plan

from dist_utils import run_distributed


def _prog(spec):
    main = static.Program()
    b = main.global_block()
    for t, ins, outs in spec:
        b.ops.append(_new(b, t, {k: [v] for k, v in ins.items()}, {"Out": [outs]}, {}))
    return b.ops


def test_stream_plan_assignment_and_minimal_waits():
    ops = _prog([("matmul_v2", {"X": "x", "Y": "w"}, "a"),        # 0 compute
                 ("c_allreduce_sum", {"X": "a"}, "b"),              # 1 comm   waits 0
                 ("relu", {"X": "x"}, "c"),                         # 2 compute (overlaps 1)
                 ("elementwise_add", {"X": "b", "Y": "c"}, "d"),    # 3 compute waits 1
                 ("c_allreduce_sum", {"X": "d"}, "e"),              # 4 comm   waits 3
                 ("scale", {"X": "e"}, "f"),                        # 5 compute waits 4
                 ("elementwise_add", {"X": "b", "Y": "f"}, "g"),    # 6 compute: 1 already covered
                 ("c_allreduce_sum", {"X": "a"}, "h")])             # 7 comm: 0 covered by pos 1's wait
    stream_of, waits, record = stream_plan(ops, list(range(len(ops))))
    assert stream_of == [0, 1, 0, 0, 1, 0, 0, 1]
    assert waits == [[], [0], [], [1], [3], [4], [], []]
    assert record == [True, True, False, True, True, False, False, False]


def test_stream_plan_war_edge():
    """A compute op overwriting a buffer a collective still reads waits for that collective."""
    ops = _prog([("c_allreduce_sum", {"X": "a"}, "b"),   # comm reads a
                 ("scale", {"X": "x"}, "a")])            # compute writes a: WAR on the comm op
    stream_of, waits, _ = stream_plan(ops, [0, 1])
    assert stream_of == [1, 0] and waits == [[], [0]]


def _tp_program(W1, W2, rank, world):
    """Row-parallel MLP as Paddle-typed ops: x · W1[:, shard] → relu → · W2[shard, :] →
    c_allreduce_sum (ring 0) → + 1 → c_allreduce_max: two collectives on the comm stream."""
    main = static.Program()
    b = main.global_block()
    n = W1.shape[1] // world
    main.params["w1"] = torch.as_tensor(W1[:, rank * n:(rank + 1) * n].copy())
    main.params["w2"] = torch.as_tensor(W2[rank * n:(rank + 1) * n].copy())
    for v in ("x", "out"):
        b.create_var(v, [None, 4])
    spec = [("matmul_v2", {"X": ["x"], "Y": ["w1"]}, {"Out": ["h"]}, {}),
            ("relu", {"X": ["h"]}, {"Out": ["r"]}, {}),
            ("matmul_v2", {"X": ["r"], "Y": ["w2"]}, {"Out": ["p"]}, {}),
            ("c_allreduce_sum", {"X": ["p"]}, {"Out": ["s"]}, {"ring_id": 0}),
            ("scale", {"X": ["s"]}, {"Out": ["t"]}, {"scale": 1.0, "bias": 1.0}),
            ("c_allreduce_max", {"X": ["t"]}, {"Out": ["out"]}, {"ring_id": 0})]
    for t, ins, outs, attrs in spec:
        b.ops.append(_new(b, t, ins, outs, attrs))
    return main


def _tp_worker(rank, world):
    r = np.random.RandomState(0)
    W1, W2, X = r.randn(4, 16).astype("float32"), r.randn(16, 4).astype("float32"), r.randn(5, 4).astype("float32")
    main = _tp_program(W1, W2, rank, world)
    exe = static.Executor("cpu")
    with static.scope_guard(static.Scope()):
        (out,) = exe.run(main, feed={"x": X}, fetch_list=["out"])
    runner = exe.last_stream_runner
    on_comm = sorted(i for i, s in runner.issued_on.items() if s == 1)
    return out, on_comm


def test_tp_program_collectives_on_comm_stream_match_serial():
    r = np.random.RandomState(0)
    W1, W2, X = r.randn(4, 16).astype("float32"), r.randn(16, 4).astype("float32"), r.randn(5, 4).astype("float32")
    ref = np.maximum(X @ W1, 0) @ W2 + 1
    res = run_distributed(_tp_worker, 2)
    for rk in range(2):
        out, on_comm = res[rk]
        assert list(on_comm) == [3, 5]
        np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)


def _dp_worker(rank, world):
    from paddle_infer_amd.static import streams
    from test_compiled_program_cpu import _train
    streams.BUCKET_MB = 1e-4  # one tiny bucket per gradient: several launches during backward
    params, losses = _train(True, rank, world)
    return params, losses


def test_dp_bucketed_overlapped_allreduce_matches_single_process():
    from test_compiled_program_cpu import _train
    ref_params, ref_losses = _train(False)
    res = run_distributed(_dp_worker, 2)
    for r in range(2):
        params, losses = res[r]
        for a, b in zip(params, ref_params):
            torch.testing.assert_close(torch.as_tensor(a), b, rtol=1e-5, atol=1e-6)
    for i, l0 in enumerate(ref_losses):
        assert (res[0][1][i] + res[1][1][i]) / 2 == pytest.approx(l0, rel=1e-5)


def test_grad_buckets_close_in_production_order():
    from paddle_infer_amd.static.streams import GradBuckets
    ops = _prog([("matmul_grad", {"X": "x"}, "w2@GRAD"), ("relu_grad", {"X": "x"}, "h"),
                 ("matmul_grad", {"X": "h"}, "w1@GRAD"), ("sgd", {"X": "w1@GRAD"}, "w1")])
    sizes = {"w2@GRAD": 3 << 20, "w1@GRAD": 1 << 20}
    gb = GradBuckets(ops, [0, 1, 2, 3], {"w1@GRAD", "w2@GRAD"}, sizes.get, bucket_mb=2)
    assert gb.buckets == [["w2@GRAD"], ["w1@GRAD"]]
    assert gb.launch_at == {0: [0], 2: [1]}


def _dp_alloc_worker(rank, world):
    from paddle_infer_amd.static import streams
    from test_compiled_program_cpu import _train
    streams.BUCKET_MB = 1e-4
    made = []
    orig = streams.GradBuckets.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        made.append(self)
    streams.GradBuckets.__init__ = init
    try:
        params, losses = _train(True, rank, world)
    finally:
        streams.GradBuckets.__init__ = orig
    return len(made), [gb.flat_allocs for gb in made], [len(gb.buckets) for gb in made], len(losses)


def test_dp_grad_buckets_persistent_flat_buffers():
    """The static DP all-reduce packs gradients into per-bucket flat buffers allocated once:
    over several training runs the allocation count stays at one per bucket (no per-step
    _flatten_dense_tensors copies), and results still match (test above)."""
    res = run_distributed(_dp_alloc_worker, 2)
    for r in range(2):
        n_plans, allocs, nb, steps = res[r]
        assert n_plans == 1 and steps > 1
        assert allocs[0] == nb[0], (allocs, nb)


def test_cpu_stream_runner_waits_on_pending_collective_inputs():
    """An op that reads the output of an earlier async all-reduce waits for that Work even when
    the plan carries no cross-stream wait for it (the gloo path has no stream ordering)."""
    from paddle_infer_amd.static.streams import StreamRunner

    class W:
        def __init__(self):
            self.done = False

        def wait(self):
            self.done = True

    class Op:
        type, func, paddle_inputs = "scale", None, None

        def __init__(self, ins):
            self.ins = ins

        def input_names(self):
            return self.ins

    r = StreamRunner(torch.device("cpu"), [1, 1], [[], []], [False, False])
    w = W()
    r.pending[0] = w
    r.pending_out[0] = {"s"}
    ran = []
    r.run(1, 1, Op(["s"]), lambda: ran.append(w.done), {})
    assert ran == [True] and not r.pending

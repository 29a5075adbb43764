"""auto_parallel planner (Strategy.auto_mode="full", reference tuner/parallel_tuner.py + cost/):
memory model calibrated on the measured single-GPU peaks, layouts that respect divisibility and the
288 GB budget, sharding / model parallelism chosen when data parallelism alone does not fit, and
Engine.plan writing the result into the Strategy."""
import pytest

from paddle_infer_amd.distributed.auto_parallel import planner as P

M1 = P.ModelSpec(24, 2048, 16, 1024, 50304)
M13 = P.ModelSpec(40, 5120, 40, 2048, 50304)
M175 = P.ModelSpec(96, 12288, 96, 2048, 50304)


def test_memory_model_matches_measurements():
    # profiles/gpt13b_1gpu_r1.txt: 223.8 GB (mb4, recompute); bench mb64 1.3B: 125.2 GB
    m13 = P.estimate(M13, P.ClusterSpec(n_gpus=1), 4, 1, 1, 1, 0, 4, True)[1] / 1e9
    m1 = P.estimate(M1, P.ClusterSpec(n_gpus=1), 64, 1, 1, 1, 0, 64, False)[1] / 1e9
    assert abs(m13 - 223.8) / 223.8 < 0.1 and abs(m1 - 125.2) / 125.2 < 0.1
    assert abs(M1.params - 1.3137e9) / 1.3137e9 < 0.01


def test_small_model_is_pure_data_parallel():
    p = P.plan(M1, P.ClusterSpec(n_gpus=8), 512)[0]
    assert (p.dp, p.tp, p.pp, p.sharding_stage) == (8, 1, 1, 0)


def test_large_models_need_sharding_or_model_parallel():
    for n, gb in ((8, 64), (64, 512)):
        p = P.plan(M175, P.ClusterSpec(n_gpus=n), gb)[0] if n == 64 else None
        if p is not None:
            assert p.sharding_stage > 0 or p.tp * p.pp > 1
            assert p.mem_gb <= 288 * 0.92
    with pytest.raises(ValueError):
        P.plan(M175, P.ClusterSpec(n_gpus=8), 64)  # 175B x 16 B/param does not fit 8 x 288 GB
    # 13B on 8 GPUs: every returned layout fits and divides the model
    for p in P.plan(M13, P.ClusterSpec(n_gpus=8), 64, top_k=5):
        assert p.mem_gb <= 288 * 0.92 and 40 % p.tp == 0 and 40 % p.pp == 0
        assert p.dp * p.tp * p.pp == 8


def test_tp_and_pp_costs_are_charged():
    c = P.ClusterSpec(n_gpus=8)
    base = P.estimate(M13, c, 64, 8, 1, 1, 1, 1, False)
    tp = P.estimate(M13, c, 64, 4, 2, 1, 1, 1, False)
    pp = P.estimate(M13, c, 64, 4, 1, 2, 1, 2, False)
    assert tp[2]["tp_comm_ms"] > 0 and tp[1] < base[1]
    assert pp[2]["bubble_ms"] > 0 and pp[1] < base[1]


def test_engine_plan_updates_strategy():
    from paddle_infer_amd.distributed.auto_parallel import Engine, Strategy
    from paddle_infer_amd.models.gpt import GPTForPretraining, gpt_config
    m = GPTForPretraining(gpt_config("gpt3-tiny"))
    st = Strategy({"auto_mode": "full"})
    eng = Engine(m, strategy=st)
    p = eng.plan(global_batch=16, n_gpus=8)
    assert st.plan is p and eng.hybrid_configs["mp_degree"] == p.tp
    assert st.amp.enable and st.pipeline.micro_batch_size == p.micro_batch

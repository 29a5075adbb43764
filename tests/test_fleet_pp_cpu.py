"""Pipeline parallelism on GPT (CPU gloo), each run matching a single-process run of the same
global batch — reference test strategy `hybrid_parallel_pp_transformer.py` /
`hybrid_parallel_pp_layer_with_virtual_stage.py`:

* pp 2 x dp 2 through fleet.init / distributed_model (GPTForPretrainingPipe → PipelineParallel,
  1F1B) / distributed_optimizer, tied embeddings shared between the first and last stage;
* pp 2 interleaved (2 virtual chunks per rank, interleaved 1F1B), untied head;
* pp 4 interleaved with 4 micro-batches (the all-warm-up corner of the schedule).
"""
import copy

import pytest
import torch

from dist_utils import run_distributed


def _cfg(layers=4, tie=True, recompute=False):
    from paddle_infer_amd.models.gpt import gpt_config
    return gpt_config("gpt3-tiny", dtype="float32", hidden_dropout_prob=0.0, num_layers=layers,
                      hidden_size=64, num_heads=4, vocab_size=128, max_position_embeddings=64,
                      tie_word_embeddings=tie, recompute=recompute)


def _data(steps=3, B=8, S=16, V=128):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, V, (B, S + 1), generator=g) for _ in range(steps)]


def _adamw(params):
    import paddle_infer_amd as paddle
    return paddle.optimizer.AdamW(learning_rate=1e-2, parameters=params, weight_decay=0.1,
                                  grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))


def _single(cfg, init, steps=3):
    from paddle_infer_amd.models.gpt import GPTForPretraining
    m = GPTForPretraining(cfg)
    m.set_state_dict(init)
    opt = _adamw(m.parameters())
    losses = []
    for ids in _data(steps):
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(loss.item())
    return {k: v.clone() for k, v in m.state_dict().items()}, losses


def _pp_worker(rank, world, init, layers, tie, pp, dp, virtual, accumulate):
    from paddle_infer_amd.distributed import fleet
    from paddle_infer_amd.models.gpt import (GPTForPretrainingPipe, gpt_pipe_load_full_state,
                                             gpt_pipe_state_to_full)
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {"dp_degree": dp, "mp_degree": 1, "pp_degree": pp, "sharding_degree": 1}
    st.pipeline_configs = {"accumulate_steps": accumulate}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    cfg = _cfg(layers, tie)
    pipe = GPTForPretrainingPipe(cfg, num_virtual_pipeline_stages=virtual)
    gpt_pipe_load_full_state(pipe, init, cfg)
    model = fleet.distributed_model(pipe)
    opt = fleet.distributed_optimizer(_adamw(pipe.parameters()))
    dpr = hcg.get_data_parallel_rank()
    losses = []
    for ids in _data():
        n = ids.shape[0] // dp
        local = ids[dpr * n:(dpr + 1) * n]
        loss = model.train_batch([local[:, :-1], local[:, 1:]], opt)
        t = loss.detach().clone().reshape(1)
        import torch.distributed as dist
        if dp > 1:
            dist.all_reduce(t, group=hcg.get_data_parallel_group())
        losses.append(t.item() / dp)
    return {"sd": gpt_pipe_state_to_full(pipe, cfg), "losses": losses}


def _check(res, ref_sd, ref_losses, world):
    merged = {}
    for r in range(world):
        assert res[r]["losses"] == pytest.approx(ref_losses, rel=1e-4, abs=1e-5), (r, res[r]["losses"])
        for k, v in res[r]["sd"].items():
            if k in merged:  # a replica (dp) or the tied embedding on two stages: identical
                torch.testing.assert_close(v, merged[k], rtol=0, atol=0)
            merged[k] = v
    assert set(merged) == set(ref_sd)
    for k in ref_sd:
        torch.testing.assert_close(merged[k], ref_sd[k], rtol=2e-3, atol=3e-4, msg=lambda m, k=k: f"{k}: {m}")


@pytest.mark.parametrize("pp,dp,virtual,accumulate,layers,tie,world", [
    (2, 2, 1, 2, 4, True, 4),     # 1F1B, pp2 x dp2, tied embeddings across first/last stage
    (2, 1, 2, 4, 4, False, 2),    # interleaved: 2 virtual chunks per rank, untied head
    (4, 1, 2, 4, 8, True, 4),     # interleaved, micro-batches == pp degree (all warm-up)
])
def test_gpt_pipeline_matches_single(pp, dp, virtual, accumulate, layers, tie, world):
    from paddle_infer_amd.models.gpt import GPTForPretraining
    cfg = _cfg(layers, tie)
    torch.manual_seed(0)
    init = copy.deepcopy(GPTForPretraining(cfg).state_dict())
    ref_sd, ref_losses = _single(cfg, init)
    res = run_distributed(_pp_worker, world, init, layers, tie, pp, dp, virtual, accumulate)
    _check(res, ref_sd, ref_losses, world)


# ------------------------------------------------------------------------------ ZeRO stage 3
def _stage3_worker(rank, world, init, tie, recompute=False, layers=2):
    from paddle_infer_amd.distributed.sharding import group_sharded_parallel
    from paddle_infer_amd.models.gpt import GPTForPretraining
    cfg = _cfg(layers, tie, recompute)
    m = GPTForPretraining(cfg)
    m.set_state_dict(init)
    model, opt, _ = group_sharded_parallel(m, _adamw(m.parameters()), "p_g_os")
    units = model.units
    # per-block units: every decoder layer is its own unit; the root's untied head is one too
    assert sum(u.name.startswith("gpt.layers.") for u in units) == cfg.num_layers
    assert any(u.name == "<root>" for u in units) == (not tie)
    losses = []
    for ids in _data():
        n = ids.shape[0] // world
        local = ids[rank * n:(rank + 1) * n]
        loss = model(local[:, :-1], labels=local[:, 1:])
        loss.backward()
        # between steps only the shards (and persistent tied table) stay resident
        opt.step()
        opt.clear_grad()
        t = loss.detach().clone()
        import torch.distributed as dist
        dist.all_reduce(t)
        losses.append(t.item() / world)
    resident = sum(p.numel() for p in m.parameters())
    sd = model.state_dict()
    return {"sd": sd, "losses": losses, "resident": resident}


@pytest.mark.parametrize("tie", [False, True])
def test_stage3_untied_head_and_clip_matches_single(tie):
    from paddle_infer_amd.models.gpt import GPTForPretraining
    cfg = _cfg(2, tie)
    torch.manual_seed(0)
    init = copy.deepcopy(GPTForPretraining(cfg).state_dict())
    ref_sd, ref_losses = _single(cfg, init)
    res = run_distributed(_stage3_worker, 2, init, tie)
    total = sum(v.numel() for v in ref_sd.values())
    for r in range(2):
        assert res[r]["losses"] == pytest.approx(ref_losses, rel=1e-4, abs=1e-5)
        for k in ref_sd:
            torch.testing.assert_close(res[r]["sd"][k], ref_sd[k], rtol=2e-3, atol=3e-4,
                                       msg=lambda m, k=k: f"{k}: {m}")
        # released blocks hold no parameter memory between steps
        assert res[r]["resident"] < (total if not tie else total) * 0.5


def test_stage3_with_recompute_matches_single():
    """ZeRO-3 + activation recompute: the recomputed forward inside backward must not prefetch a
    block whose backward already ran (that gather would survive the optimizer step and feed the
    NEXT forward pre-step weights). 3 layers so a middle block has both neighbours."""
    from paddle_infer_amd.models.gpt import GPTForPretraining
    cfg = _cfg(3, False)
    torch.manual_seed(0)
    init = copy.deepcopy(GPTForPretraining(cfg).state_dict())
    ref_sd, ref_losses = _single(cfg, init)
    res = run_distributed(_stage3_worker, 2, init, False, True, 3)
    for r in range(2):
        assert res[r]["losses"] == pytest.approx(ref_losses, rel=1e-4, abs=1e-5)
        for k in ref_sd:
            torch.testing.assert_close(res[r]["sd"][k], ref_sd[k], rtol=2e-3, atol=3e-4,
                                       msg=lambda m, k=k: f"{k}: {m}")


# ------------------------------------------------------------- ZeRO stage 3 x pipeline (config 5)
def _pp_stage3_worker(rank, world, init, layers, tie, pp, sh, dp, accumulate, recompute, offload):
    import torch.distributed as dist
    from paddle_infer_amd.distributed import fleet
    from paddle_infer_amd.models.gpt import (GPTForPretrainingPipe, gpt_pipe_load_full_state,
                                             gpt_pipe_state_to_full)
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {"dp_degree": dp, "mp_degree": 1, "pp_degree": pp, "sharding_degree": sh}
    st.sharding_configs = {"stage": 3, "offload": offload}
    st.pipeline_configs = {"accumulate_steps": accumulate}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    cfg = _cfg(layers, tie)
    pipe = GPTForPretrainingPipe(cfg, recompute_interval=1 if recompute else 0)
    gpt_pipe_load_full_state(pipe, init, cfg)
    full_numel = sum(p.numel() for p in pipe.parameters())
    model = fleet.distributed_model(pipe)
    opt = fleet.distributed_optimizer(_adamw(pipe.parameters()))
    s3 = model._stage3
    assert sum(u.name.startswith("_stage_layers.") for u in s3.units) >= layers // pp
    # data axis = dp x sharding replicas of this stage
    drank = hcg.get_data_parallel_rank() * sh + hcg.get_sharding_parallel_rank()
    nrep = dp * sh
    losses = []
    for ids in _data():
        n = ids.shape[0] // nrep
        local = ids[drank * n:(drank + 1) * n]
        loss = model.train_batch([local[:, :-1], local[:, 1:]], opt)
        t = loss.detach().clone().reshape(1)
        dist.all_reduce(t)  # every rank holds its replica's loss: mean over all ranks
        losses.append(t.item() / world)
    resident = sum(p.numel() for p in pipe.parameters())
    s3.get_all_parameters()
    sd = gpt_pipe_state_to_full(pipe, cfg)
    s3.release_all()
    return {"sd": sd, "losses": losses, "resident": resident, "full": full_numel}


@pytest.mark.parametrize("pp,sh,dp,tie,recompute,offload", [
    (2, 2, 1, True, False, False),   # BASELINE config 5 shape: sharding stage 3 x pp 2, tied head
    (2, 2, 1, False, True, True),    # + recompute inside the stage, offloaded optimizer states
])
def test_pp_x_sharding_stage3_matches_single(pp, sh, dp, tie, recompute, offload):
    from paddle_infer_amd.models.gpt import GPTForPretraining
    layers, world = 4, pp * sh * dp
    cfg = _cfg(layers, tie)
    torch.manual_seed(0)
    init = copy.deepcopy(GPTForPretraining(cfg).state_dict())
    ref_sd, ref_losses = _single(cfg, init)
    res = run_distributed(_pp_stage3_worker, world, init, layers, tie, pp, sh, dp, 2, recompute, offload)
    _check(res, ref_sd, ref_losses, world)
    for r in range(world):  # between steps a stage holds its shards + persistent (shared) tables
        assert res[r]["resident"] < res[r]["full"], res[r]


def _dp_sharding_stage3_worker(rank, world, init, dp, sh):
    """Fleet ZeRO-3 over the sharding axis with a data-parallel axis replicating it."""
    import torch.distributed as dist
    from paddle_infer_amd.distributed import fleet
    from paddle_infer_amd.models.gpt import GPTForPretraining
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {"dp_degree": dp, "mp_degree": 1, "pp_degree": 1, "sharding_degree": sh}
    st.sharding_configs = {"stage": 3}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    cfg = _cfg(2, True)
    net = GPTForPretraining(cfg)
    net.set_state_dict(init)
    model = fleet.distributed_model(net)
    opt = fleet.distributed_optimizer(_adamw(net.parameters()))
    assert type(model).__name__ == "GroupShardedStage3" and model.world == sh
    drank = hcg.get_data_parallel_rank() * sh + hcg.get_sharding_parallel_rank()
    losses = []
    for ids in _data():
        n = ids.shape[0] // world
        local = ids[drank * n:(drank + 1) * n]
        loss = model(local[:, :-1], labels=local[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        t = loss.detach().clone()
        dist.all_reduce(t)
        losses.append(t.item() / world)
    return {"sd": model.state_dict(), "losses": losses}


def test_dp_x_sharding_stage3_matches_single():
    from paddle_infer_amd.models.gpt import GPTForPretraining
    cfg = _cfg(2, True)
    torch.manual_seed(0)
    init = copy.deepcopy(GPTForPretraining(cfg).state_dict())
    ref_sd, ref_losses = _single(cfg, init)
    res = run_distributed(_dp_sharding_stage3_worker, 4, init, 2, 2)
    _check(res, ref_sd, ref_losses, 4)

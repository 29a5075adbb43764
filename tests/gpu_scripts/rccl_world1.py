"""Child process of tests/test_rccl_world1_gpu.py: a 1-rank RCCL ("nccl") process group created
before any other GPU call, then the data / tensor-parallel engines run with their collectives
FORCED on (PIAMD_FORCE_COLLECTIVES=1) — flat-engine ZeRO-1 (reduce-scatter hooks + parameter
all-gather), DataParallel (bucketed async all-reduce), TP column/row-parallel layers (async dX
all-reduce, output all-reduce) and the static data-parallel GradBuckets — then the same runs
without a process group. Prints one JSON line of per-path losses (with, without)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CPU = os.environ.get("PIAMD_TEST_DEVICE") == "cpu"  # dry run of this script without a GPU (gloo)
dev = torch.device("cpu") if CPU else torch.device("cuda", 0)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
if CPU:
    dist.init_process_group("gloo", rank=0, world_size=1)
else:
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)  # first GPU call of the process
    torch.cuda.set_device(dev)

import numpy as np  # noqa: E402

import paddle_infer_amd as paddle  # noqa: E402
from paddle_infer_amd import static  # noqa: E402


def mlp(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.GELU(), torch.nn.Linear(128, 32)).to(dev)


def data(seed, n=2):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [(torch.randn(16, 64, generator=g).to(dev), torch.randn(16, 32, generator=g).to(dev)) for _ in range(n)]


def run_flat(group):
    from paddle_infer_amd.parallel.flat_engine import FlatTrainer
    m = mlp(1)
    eng = FlatTrainer(m, lr=1e-2, dp_group=group, sharding_stage=1, bucket_mb=1, grad_clip=None)
    out = []
    for x, y in data(2):
        loss = ((m(x) - y) ** 2).mean()
        loss.backward()
        eng.step()
        eng.zero_grad()
        out.append(loss.item())
    eng.wait_params()
    out.append(sum(float(p.detach().double().sum()) for p in m.parameters()))
    run_flat.sharding = eng.sharding  # 1 only when the ZeRO-1 collectives ran
    return out


def run_dp(group):
    from paddle_infer_amd.distributed.parallel import DataParallel
    m = mlp(3)
    dp = DataParallel(m, group=group, comm_buffer_size=1) if group is not None else m
    opt = torch.optim.SGD(m.parameters(), lr=0.05)
    out = []
    for x, y in data(4):
        loss = ((dp(x) - y) ** 2).mean()
        loss.backward()
        if group is not None and hasattr(dp, "_finish"):
            dp._finish()
        opt.step()
        opt.zero_grad(set_to_none=False)
        out.append(loss.item())
    return out


def run_tp(group):
    from paddle_infer_amd.distributed.fleet.mp_layers import ColumnParallelLinear, RowParallelLinear
    torch.manual_seed(5)
    c = ColumnParallelLinear(64, 128, gather_output=False, mp_group=group).to(dev)
    r = RowParallelLinear(128, 32, input_is_parallel=True, mp_group=group).to(dev)
    params = list(c.parameters()) + list(r.parameters())
    opt = torch.optim.SGD(params, lr=0.05)
    out = []
    for x, y in data(6):
        x = x.requires_grad_(True)
        loss = ((r(torch.relu(c(x))) - y) ** 2).mean()
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        out.append(loss.item())
        out.append(float(x.grad.double().sum()))
    return out


def run_static(forced):
    paddle.enable_static()
    try:
        torch.manual_seed(7)
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data("x", [None, 8], "float32")
            y = static.data("y", [None, 1], "float32")
            h = static.nn.fc(x, 16, activation="relu")
            pred = static.nn.fc(h, 1)
            loss = paddle.mean((pred - y) ** 2)
            paddle.optimizer.SGD(learning_rate=0.1).minimize(loss)
        exe = static.Executor("cpu" if CPU else "gpu")
        bs = static.BuildStrategy()
        bs.fuse_all_reduce_ops = True
        prog = static.CompiledProgram(main, build_strategy=bs).with_data_parallel(loss_name=loss.var_name)
        r = np.random.RandomState(1)
        out, plans = [], None
        with static.scope_guard(static.Scope()):
            for _ in range(2):
                (lv,) = exe.run(prog, feed={"x": r.randn(8, 8).astype("float32"),
                                            "y": r.randn(8, 1).astype("float32")}, fetch_list=[loss])
                out.append(float(lv))
            plans = [k for k in getattr(exe, "_plans", {}) if isinstance(k, tuple) and k and k[0] == "dp_buckets"]
        return out, len(plans)
    finally:
        paddle.disable_static()


res = {}
os.environ["PIAMD_FORCE_COLLECTIVES"] = "1"
W = dist.group.WORLD
res["flat"] = [run_flat(W)]
res["flat_sharding_forced"] = run_flat.sharding
res["dp"] = [run_dp(W)]
res["tp"] = [run_tp(W)]
s_out, s_plans = run_static(True)
res["static"] = [s_out]
res["static_bucket_plans"] = s_plans
if not CPU:
    torch.cuda.synchronize()
dist.destroy_process_group()
os.environ["PIAMD_FORCE_COLLECTIVES"] = "0"
res["flat"].append(run_flat(None))
res["dp"].append(run_dp(None))
res["tp"].append(run_tp(None))
res["static"].append(run_static(False)[0])
print("RESULT " + json.dumps(res))
sys.stdout.flush()

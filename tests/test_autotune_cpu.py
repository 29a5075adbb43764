"""Runtime plan autotuning (ops/autotune.py, reference phi/kernels/autotune): heuristic outside
the tuning range, measured winner inside it (cached per key, persisted to / replayed from a JSON
cache file), and the optimizer advancing the step counter."""
import json

import torch

from paddle_infer_amd.ops import autotune as AT


def _reset():
    AT.CACHE.clear()
    AT._STATE.update({"enable": False, "range": (0, 1 << 62), "step": 0, "cache_file": None})


def test_choose_heuristic_then_tuned(monkeypatch, tmp_path):
    _reset()
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    cost = {(64, 1): 3.0, (128, 2): 1.0, (256, 4): 2.0}
    monkeypatch.setattr(AT, "_time", lambda run, plan: cost[plan])
    ran = []
    key = AT.key_of("conv2d_fwd", 2, 16, 16, 64)
    assert AT.choose(key, list(cost), (64, 1), ran.append) == (64, 1)  # tuning off
    assert not ran
    cache = tmp_path / "tune.json"
    AT.configure(enable=True, tuning_range=[2, 5], cache_file=str(cache))
    assert AT.choose(key, list(cost), (64, 1), ran.append) == (64, 1)  # step 0 < 2
    AT.step(), AT.step()
    assert AT.choose(key, list(cost), (64, 1), ran.append) == (128, 2)
    assert set(ran) == set(cost)
    assert json.loads(cache.read_text())[key] == [128, 2]
    ran.clear()
    assert AT.choose(key, list(cost), (64, 1), ran.append) == (128, 2) and not ran  # cached
    _reset()
    AT.configure(enable=False, cache_file=str(cache))  # a new process replays the file
    assert AT.choose(key, list(cost), (64, 1), ran.append) == (128, 2)
    _reset()


def test_optimizer_step_advances_counter():
    _reset()
    import paddle_infer_amd as paddle
    p = torch.nn.Parameter(torch.ones(3))
    opt = paddle.optimizer.SGD(learning_rate=0.1, parameters=[p])
    p.grad = torch.ones(3)
    opt.step()
    opt.step()
    assert AT._STATE["step"] == 2
    _reset()

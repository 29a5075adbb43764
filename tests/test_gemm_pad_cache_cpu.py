"""ops.gemm._kc: a weight's zero-padded K-contiguous image is cached (keyed by version and the
parameter epoch) and refreshed when the weight changes; activations are never cached."""
import torch

from paddle_infer_amd.ops import gemm as G
from paddle_infer_amd.ops import linear as L


def test_padded_weight_cached_and_invalidated():
    w = torch.nn.Parameter(torch.randn(10, 70).bfloat16())
    a = G._kc(w, 128, 16, cache=True)
    assert G._kc(w, 128, 16, cache=True) is a
    assert a.shape == (16, 128) and torch.equal(a[:10, :70], w.detach()) and a[10:].abs().sum() == 0
    with torch.no_grad():
        w.add_(1)  # version bump
    b = G._kc(w, 128, 16, cache=True)
    assert b is not a and torch.equal(b[:10, :70], w.detach())
    L.bump_param_epoch()  # raw-pointer optimizer write
    assert G._kc(w, 128, 16, cache=True) is not b


def test_activation_not_cached():
    x = torch.randn(10, 70).bfloat16()
    assert G._kc(x, 128, 16, cache=True) is not G._kc(x, 128, 16, cache=True)
    assert not hasattr(x, "_piamd_pad")

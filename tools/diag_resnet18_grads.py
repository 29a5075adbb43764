"""Per-parameter gradient cosines of a ResNet-18 bf16 step: library conv (twice), HIP conv and an
fp32 library run (the common reference). Usage: python tools/diag_resnet18_grads.py"""
import torch, torch.nn.functional as F, sys
sys.path.insert(0, '.')
import paddle_infer_amd
from paddle_infer_amd.ops import conv as CV
from paddle_infer_amd.vision.models import resnet18
DEV='cuda'
torch.manual_seed(0)
m = resnet18(num_classes=10).to(DEV).to(memory_format=torch.channels_last)
x = torch.randn(16, 3, 64, 64, device=DEV).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (16,), device=DEV)
res = {}
for tag, hc in (("lib", False), ("lib2", False), ("hip", True), ("fp32", False)):
    CV.HIP_CONV = hc
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=tag != "fp32"):
        loss = F.cross_entropy(m(x), y)
    loss.backward()
    res[tag] = (loss.item(), [(n, p.grad.float().flatten().clone()) for n, p in m.named_parameters()])
print("loss", res["lib"][0], res["lib2"][0], res["hip"][0], res["fp32"][0])
cs = lambda a, b: F.cosine_similarity(a, b, dim=0).item()
for (n, a), (_, b), (_, c), (_, f) in zip(res["lib"][1], res["lib2"][1], res["hip"][1], res["fp32"][1]):
    print(f"{n:32s} lib/lib2 {cs(a,b):.4f} lib/hip {cs(a,c):.4f} lib/fp32 {cs(a,f):.4f} hip/fp32 {cs(c,f):.4f}")

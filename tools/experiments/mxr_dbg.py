import sys, torch
sys.path.insert(0, '.')
from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref
sys.path.insert(0, 'tests')
from test_mx_gpu import _act, _weights, DEV
K, N, eps = 1024, 256, 1e-5
M = 48
x = (_act(M, K, 5, spread=False).float() * 3).to(torch.bfloat16).to(DEV)
act = ops.quantize_act_mx(x)
xa = ref.dequant_mx(act.q.cpu(), act.e.cpu())
inv = torch.rsqrt(xa.pow(2).mean(-1, keepdim=True) + eps)
wq = _weights(N, K, 23)
raw = xa @ ref.dequant_fp8(wq.q.cpu(), wq.scale.cpu()).t()
for cfg in range(len(ops.mgemm_configs())):
    if not ops.mgemm_valid(cfg, M, N, K, ops.EPI_BF16, 3):
        continue
    y = ops.mgemm(act, wq, ops.EPI_BF16, cfg=cfg, grid=1, rms_eps=eps).float().cpu()
    ratio = (y / raw).median(dim=1).values          # = the kernel's 1 / rms per row
    r = (ratio / inv[:, 0]) ** -2                     # kernel's sum of squares / true
    print(cfg, ops.mgemm_configs()[cfg], 'sumsq ratio per row (first 4, min, max):', [round(v, 3) for v in r[:4].tolist()], round(r.min().item(), 3), round(r.max().item(), 3), flush=True)

import sys, time, torch
sys.path.insert(0, ".")
from k8s_llm_scheduler_amd.engine import _load_gemm_table
sys.path.insert(0, "tools")
from kbench import timeit
x = torch.randn(64, 28672, device="cuda", dtype=torch.bfloat16)
w = torch.randn(8192, 28672, device="cuda", dtype=torch.bfloat16) * 0.02
f = lambda: torch.nn.functional.linear(x, w)
print("default", timeit(f, 50))
print("loaded", _load_gemm_table(), torch.cuda.tunable.is_enabled(), torch.cuda.tunable.tuning_is_enabled())
print("table", timeit(f, 50))
f(); torch.cuda.synchronize()
t0=time.perf_counter()
for _ in range(50): f()
torch.cuda.synchronize(); print("eager table", (time.perf_counter()-t0)/50*1e6)

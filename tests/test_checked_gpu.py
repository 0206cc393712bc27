"""Bounds-checked kernel build (K8S_CHECKED=1, ``ops/_C_checked*.so``; SURVEY.md section 5 "bounds asserts in kernel
debug builds"): with valid inputs the checked kernels record nothing and match the release kernels bit for bit; a
corrupted block table, slot mapping or token id is recorded (unit, line, value) and its index clamped, so the kernel
finishes without touching memory it does not own, and the engine step raises KernelCheckError.

Runs in a child process: the extension variant is chosen when ``ops`` is imported."""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import sys, torch
sys.path.insert(0, ROOT)
from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.models.config import PRESETS
from k8s_llm_scheduler_amd.models.llama import LlamaModel
assert ops.CHECKED and ops.native().checked, "the checked extension is not the one loaded"
dev = torch.device("cuda")
m = LlamaModel(PRESETS["tiny"], device="cuda", seed=1, max_model_len=256)
m.allocate_kv(9, 16)                       # 9 blocks, 144 slots: the bounds the checked kernels enforce
nq, nkv, D = m.nq, m.nkv, m.D
kc, vc = m.kv_cache[0, 0], m.kv_cache[0, 1]
g = torch.Generator(device="cpu").manual_seed(0)
qkv = (torch.randn(2, (nq + 2 * nkv) * D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
ctx = torch.tensor([20, 40], dtype=torch.int32, device=dev)
bt = torch.tensor([[0, 1, 2, 3], [4, 5, 6, 7]], dtype=torch.int32, device=dev)

def run_decode(split, bt_):
    keep = ops.SPLIT_MAX_PAIRS
    ops.SPLIT_MAX_PAIRS = 64 if split else 0
    try:
        kc.zero_(); vc.zero_()
        y = ops.decode_attention_fused(qkv, m.cos_sin, kc, vc, bt_, ctx, m.scale, 16, 64, nq, nkv, D)
    finally:
        ops.SPLIT_MAX_PAIRS = keep
    torch.cuda.synchronize()
    return y

for split in (True, False):
    y = run_decode(split, bt)
    assert ops.check_read(dev) is None, f"valid inputs flagged (split={split})"
    bad = bt.clone(); bad[1, 1] = 1000           # a block id past the cache (row 1's second block)
    run_decode(split, bad)
    v = ops.check_read(dev)
    assert v is not None and v["code"] == 2 and v["value"] == 1000, v
    assert v["where"] == ("attn_decode_split.hip" if split else "attn_decode_fused.hip"), v
    print("decode", "split" if split else "fused", v["count"], "violations, first at line", v["line"])

# prefill KV write with a slot past the cache: recorded, the token's K/V not written
pos = torch.tensor([0, 1], dtype=torch.int32, device=dev)
slots = torch.tensor([5, 999], dtype=torch.int32, device=dev)
kc.zero_()
ops.rope_kv_write(qkv, m.cos_sin, kc, vc, nq, nkv, D, positions=pos, slot_mapping=slots)
torch.cuda.synchronize()
v = ops.check_read(dev)
assert v is not None and v["code"] == 1 and v["value"] == 999 and v["where"] == "rope_kv.hip", v
assert float(kc[5].abs().sum()) > 0, "the valid slot was not written"
print("rope_kv slot", v)

# prefill attention over a block table with a bad id
q = (torch.randn(24, nq, D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
cu = torch.tensor([0, 24], dtype=torch.int32, device=dev)
pctx = torch.tensor([40], dtype=torch.int32, device=dev)
pbt = torch.tensor([[0, 1, 2, 3]], dtype=torch.int32, device=dev)
ops.paged_prefill_attention(q, kc, vc, cu, pctx, pbt, m.scale, 16, 24)
torch.cuda.synchronize()
assert ops.check_read(dev) is None
pbt[0, 2] = -7
ops.paged_prefill_attention(q, kc, vc, cu, pctx, pbt, m.scale, 16, 24)
torch.cuda.synchronize()
v = ops.check_read(dev)
assert v is not None and v["code"] == 2 and v["value"] == -7 and v["where"] == "attn_prefill.hip", v
print("prefill attention", v)

# token id past the vocabulary
e = ops.embedding(torch.tensor([3, 10 ** 6], dtype=torch.int32, device=dev), m.embed)
torch.cuda.synchronize()
v = ops.check_read(dev)
assert v is not None and v["code"] == 4 and v["value"] == 10 ** 6, v
try:
    ops.embedding(torch.tensor([10 ** 6], dtype=torch.int32, device=dev), m.embed)
    ops.check_raise(dev)
    raise AssertionError("check_raise did not raise")
except ops.KernelCheckError as err:
    print("raised:", err)
print("CHECKED-OK")
"""


def test_checked_kernels_record_and_clamp_bad_indices():
    so = os.path.join(ROOT, "k8s_llm_scheduler_amd", "ops")
    if not any(f.startswith("_C_checked") and f.endswith(".so") for f in os.listdir(so)):
        pytest.fail("ops/_C_checked*.so missing: python -m k8s_llm_scheduler_amd._build --checked")
    env = dict(os.environ, K8S_CHECKED="1", PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + PROBE], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0 and "CHECKED-OK" in p.stdout, (p.stdout[-3000:], p.stderr[-3000:])


def test_checked_engine_step_raises_kernel_check_error():
    """A whole engine (tiny model, captured graphs) on the checked build decides normally; a block-table entry
    corrupted behind the engine's back makes the next step raise KernelCheckError.  (This run faulted while the
    violation recorder was a non-inlined device function called from the graph-captured split-attention kernel; the
    recorder is inlined since.)"""
    code = r"""
import sys, torch
sys.path.insert(0, ROOT)
from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
eng = build_engine("tiny", device="cuda", max_batch=2, max_model_len=256, num_blocks=32, seed=1)
outs = eng.generate([[7, 100, 2000, 31, 32, 33]], SamplingParams(max_tokens=6, temperature=0.0))
assert len(outs[0].token_ids) == 6, outs
r = eng.add_request([7, 100, 2000, 31, 32, 33, 5, 5], SamplingParams(max_tokens=40, temperature=0.0))
eng.step()                                       # prefill + first decode chunk
eng.s_bt[r.slot, 0] = 10 ** 5                    # corrupt the running request's first block id
try:
    for _ in range(10):
        eng.step()
    raise AssertionError("no KernelCheckError")
except ops.KernelCheckError as e:
    print("raised:", e)
print("ENGINE-CHECKED-OK")
"""
    env = dict(os.environ, K8S_CHECKED="1", PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0 and "ENGINE-CHECKED-OK" in p.stdout, (p.stdout[-3000:], p.stderr[-3000:])

"""Host-side cost per call of the drop-in interface (tiny inputs, GPU time negligible)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn import flash_attn_hip as hip  # noqa: E402
from flash_attn.flash_attn_interface import flash_attn_unpadded_func  # noqa: E402

q = torch.randn(64, 2, 64, device="cuda", dtype=torch.bfloat16)
cu = torch.tensor([0, 64], dtype=torch.int32, device="cuda")
for fn, name in ((lambda: flash_attn_unpadded_func(q, q, q, cu, cu, 64, 64, 0.0), "interface"),
                 (lambda: hip.fwd(q, q, q, cu, cu, 64, 64, 0.0, 0.125, False, False, False, None), "hip.fwd")):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2000):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t) / 2000 * 1e6:.1f} us/call")
pr = cProfile.Profile()
pr.enable()
for _ in range(2000):
    flash_attn_unpadded_func(q, q, q, cu, cu, 64, 64, 0.0)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(15)

"""Wall time per call of the north-star forward through each layer of the stack, back to back:
the drop-in interface, flash_attn_hip.fwd, and a bare ctypes fa_fwd on preallocated buffers;
plus HIP-event time over the same loops. Shows where `value` (wall) and the kernel time part."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn import flash_attn_hip as hip  # noqa: E402
from flash_attn.flash_attn_interface import flash_attn_unpadded_func  # noqa: E402

B, H, S, D = 8, 12, 2048, 64
g = torch.Generator().manual_seed(0)
q, k, v = (torch.randn(B * S, H, D, generator=g).bfloat16().cuda() for _ in range(3))
cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device="cuda")
o = torch.empty_like(q)
lse = torch.empty(B, H, S, dtype=torch.float32, device="cuda")
a = hip.FaFwdArgs()
a.q, a.k, a.v, a.o, a.softmax_lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr()
a.cu_seqlens_q = a.cu_seqlens_k = cu.data_ptr()
for n in ("q", "k", "v", "o"):
    setattr(a, f"{n}_row_stride", H * D)
    setattr(a, f"{n}_head_stride", D)
a.batch, a.nheads, a.head_dim, a.max_seqlen_q, a.max_seqlen_k, a.lse_stride = B, H, D, S, S, S
a.softmax_scale, a.dtype = D ** -0.5, hip.FA_DTYPE_BF16
L = hip.lib()
st = torch.cuda.current_stream().cuda_stream
fns = {
    "interface": lambda: flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0),
    "hip.fwd": lambda: hip.fwd(q, k, v, cu, cu, S, S, 0.0, D ** -0.5, False, False, False, None),
    "ctypes": lambda: L.fa_fwd(ctypes.byref(a), st),
}
flops = 4.0 * B * H * S * S * D
for rnd in range(2):
    for name, fn in fns.items():
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(200):
            fn()
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 200 * 1e3
        ev = e0.elapsed_time(e1) / 200
        print(f"round {rnd} {name:10s} wall {wall:.4f} ms ({flops / wall / 1e9:.0f} TF)  events {ev:.4f} ms", flush=True)

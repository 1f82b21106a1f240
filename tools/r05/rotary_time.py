import sys, torch
sys.path.insert(0, "hazyresearch_flash-attention_amd")
from flash_attn.rotary import RotaryEmbedding, apply_rotary_emb_qkv_
dev = torch.device("cuda")
qkv = torch.randn(8, 2048, 3 * 12 * 64, generator=torch.Generator().manual_seed(5)).bfloat16().to(dev)
rc, rs = RotaryEmbedding(64).to(dev).cos_sin_tables(2048, dev, torch.bfloat16)
for _ in range(20): apply_rotary_emb_qkv_(qkv, rc, rs, 12, 64)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200): apply_rotary_emb_qkv_(qkv, rc, rs, 12, 64)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 200
print("rotary inplace ms", round(ms, 4), "frac_hbm", round(2*2*8*2048*12*64*2/ms/1e6/8000, 3))

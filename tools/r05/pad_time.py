"""Time the var-len gather / zero-filling scatter of bench.py's extra (tools only)."""
import sys
import torch
sys.path.insert(0, "hazyresearch_flash-attention_amd")
sys.path.insert(0, ".")
from flash_attn.bert_padding import index_first_axis, index_put_first_axis  # noqa: E402
from oracle.attention_ref import generate_random_padding_mask  # noqa: E402
dev = torch.device("cuda")
hs = torch.randn(8 * 2048, 12, 64, generator=torch.Generator().manual_seed(3)).bfloat16().to(dev)
pm = generate_random_padding_mask(2048, 8, "cpu", "third", generator=torch.Generator().manual_seed(4))
pidx = torch.nonzero(pm.reshape(-1)).reshape(-1).to(dev)
packed = index_first_axis(hs, pidx)
for name, fn in (("gather", lambda: index_first_axis(hs, pidx)), ("scatter", lambda: index_put_first_axis(packed, pidx, 8 * 2048))):
    for _ in range(20): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200): fn()
    e1.record(); torch.cuda.synchronize()
    print(name, "event ms", round(e0.elapsed_time(e1) / 200, 4), "rows", pidx.numel())

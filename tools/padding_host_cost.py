"""Host vs device time of the bert_padding row moves (tools only): per call, the HIP-event time of
back-to-back interface calls, the device time of the same calls replayed from a HIP graph, and the
host enqueue time (perf_counter over calls without device waits), for index_first_axis (unpad gather)
and index_put_first_axis (pad scatter) at bench.py's shape.

    python tools/padding_host_cost.py > gpurun_out/padding_host_cost.txt
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from flash_attn.bert_padding import index_first_axis, index_put_first_axis  # noqa: E402
from oracle.attention_ref import generate_random_padding_mask  # noqa: E402
import bench  # noqa: E402


def host_us(fn, n=2000):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return host


def main():
    dev = torch.device("cuda")
    hs = torch.randn(8 * 2048, 12, 64, generator=torch.Generator().manual_seed(3)).bfloat16().to(dev)
    pm = generate_random_padding_mask(2048, 8, "cpu", "third", generator=torch.Generator().manual_seed(4))
    pidx = torch.nonzero(pm.reshape(-1)).reshape(-1).to(dev)
    packed = index_first_axis(hs, pidx)
    for name, fn in (("unpad_gather", lambda: index_first_axis(hs, pidx)),
                     ("pad_scatter", lambda: index_put_first_axis(packed, pidx, 8 * 2048))):
        ev, _ = bench.time_events(fn, 200, 20)
        gr = bench.graph_ms(fn, 50)
        print(json.dumps({"op": name, "event_us_per_call": round(ev * 1e3, 2),
                          "graph_us_per_call": round(gr * 1e3, 2) if gr else None,
                          "host_enqueue_us_per_call": round(host_us(fn), 2)}), flush=True)


if __name__ == "__main__":
    main()

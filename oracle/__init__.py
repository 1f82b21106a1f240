"""CPU oracle for the FlashAttention hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker (or the timed CPU baseline), never as the product path. The product
(flash_attn.flash_attn_hip -> libfa_hip.so) has no CPU fallback.

Pinning: attention_ref.py is checked against golden vectors produced by the
reference's own `attention_ref` (tests/golden/make_golden.py); philox.py against the Random123
Philox-4x32-10 known-answer vectors; fa_tiled.c (the tiled online-softmax restatement) against
attention_ref.py.
"""

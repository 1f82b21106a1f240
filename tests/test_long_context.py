"""GPU parity at the BASELINE.json C4 size and at long context (the reference claims it "can
scale up to sequence length 64K", README.md:75).

These run the launch paths that only long sequences reach: the causal LPT block order of the
forward and backward, the D=128 P/dS split backward with its query-major dQ pass (dense) or its
fp32 dQ atomics (dropout), and 16K-key walks. Each case is checked against the fp32 oracle with
the reference's 2x rule (tests/test_flash_attn.py:407-409) on outputs, attention probabilities
and dQ/dK/dV (run_case in test_flash_attn.py), at batch/head counts the oracle finishes in a few
seconds on the GPU.
"""
import pytest
import torch

from test_flash_attn import run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("causal", [True, False])
def test_c4_shape_d128_s4096(causal):
    """C4 (B16 H12 S4096 D128 bf16 causal) at B=2 H=2: split backward + query-major dQ pass."""
    run_case("separate", 2, 4096, 4096, 2, 128, torch.bfloat16, causal, 0.0, mode="full")


def test_c4_shape_d128_s4096_dropout():
    """D=128 with dropout at S=4096: the split kernel's fp32 dQ atomics over 32 key blocks."""
    run_case("separate", 2, 4096, 4096, 2, 128, torch.bfloat16, True, 0.1, mode="full")


@pytest.mark.parametrize("d", [64, 128])
def test_c4_ragged_s4096(d):
    """Random padding at S=4096 (varlen cu_seqlens, partial last tiles, LPT order with short rows)."""
    run_case("qkvpacked", 2, 4096, 4096, 2, d, torch.bfloat16, True, 0.0)


def test_long_context_s16384_d64_causal():
    """S=16384, D=64, causal, B=1 H=1: 256-key tiles x 64 query blocks, 16K-key walks."""
    run_case("separate", 1, 16384, 16384, 1, 64, torch.bfloat16, True, 0.0, mode="full")


def test_long_context_s8192_d64_dropout_fp16():
    """S=8192 fp16 causal with dropout (atomic-dQ D=64 backward over 32 key blocks)."""
    run_case("separate", 1, 8192, 8192, 2, 64, torch.float16, True, 0.1, mode="full")


@pytest.mark.parametrize("causal", [False, True])
def test_forward_grid_balance_four_wave_workgroups(causal):
    """B=1 H=36 S=2048: 288 eight-wave workgroups, between one and two per CU of a 256-CU device,
    so the launcher picks 4-wave workgroups (fa_kernels_impl.h pick_fwd_waves) without dropout."""
    run_case("separate", 1, 2048, 2048, 36, 64, torch.bfloat16, causal, 0.0)


@pytest.mark.parametrize("seqlen_k,mode", [(1, "full"), (63, "full"), (65, "full"), (130, "random"), (4095, "random")])
def test_forward_split_k_key_halves(seqlen_k, mode):
    """Small grids take the intra-workgroup split-K forward (two key groups per 128-row block,
    merged through LDS). Key counts where the second group gets no key (1, 63), one partial tile
    (65, 130) or a long walk (4095); random padding where the mask generator allows it. With one
    key the exact dQ is 0 (dP = delta), which the 2x rule cannot bound, so that case checks the
    forward only (the 1-key backward is covered by test_empty_and_ragged_sequences_backward)."""
    run_case("kvpacked", 2, 300, seqlen_k, 2, 64, torch.bfloat16, False, 0.0, mode=mode, grad=seqlen_k > 1)

"""MI355X-native FlashAttention (drop-in for the reference's `flash_attn` package).

Add `hazyresearch_flash-attention_amd/` to sys.path and import as before:
    from flash_attn.flash_attn_interface import flash_attn_unpadded_func
"""
__version__ = "0.1.0"

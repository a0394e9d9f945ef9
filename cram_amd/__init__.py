"""cram_amd — MI355X-native credibility-aware attention (CrAM hot path).

Drop-in for /root/reference/utils/re_weighting.py: the dense-mask forward-pre-hook
is replaced by fused gfx950 HIP attention kernels behind a C-ABI
(include/cram_attn.h), registered with transformers' AttentionInterface.
"""
__version__ = "0.1.0"

"""eegfusion — MI355X-native (gfx950) fusion training path of Rachfu/EEG-multimodal.

Host-side Python over the C-ABI library ``libeegfusion.so`` (hand-written HIP kernels).
"""
__all__ = ["kernels"]

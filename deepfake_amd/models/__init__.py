"""nn.Module surface of /root/reference/src/models on the MI355X path."""
import torch


def set_compute_dtype(model, dtype):
    """Activation / weight compute dtype for every module that creates activations
    from raw inputs (patch embeddings, the waveform front end)."""
    for m in model.modules():
        if hasattr(m, "compute_dtype"):
            m.compute_dtype = dtype
    return model


def set_fp8(model, stages=(2, 3)):
    """C4's fp8 path (BASELINE configs[3]): the qkv / proj / fc1 / fc2 GEMMs of the Video Swin blocks in `stages`
    (0-based) run forward and input gradient on MX-fp8 operands (dfk_gemm_mx); the weight gradients, attention and
    everything else stay bf16.  Default: stages 3 and 4, whose Linears are MFMA-bound — stages 1-2 (K <= 512 over
    401k / 100k tokens) stream HBM, where the extra quantisation pass costs more than the faster MFMA saves
    (profiles/fp8/r4d_mx_vs_bf16_gemm_bench.txt).  Returns the number of blocks switched."""
    from .video_swin_transformer import SwinTransformer3D
    n = 0
    for m in model.modules():
        if isinstance(m, SwinTransformer3D):
            for i, layer in enumerate(m.layers):
                for blk in layer.blocks:
                    blk.mx = i in stages
                    n += int(blk.mx)
    return n


__all__ = ["set_compute_dtype", "set_fp8", "torch"]

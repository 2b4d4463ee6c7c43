"""nn.Module surface of /root/reference/src/models on the MI355X path."""
import torch


def set_compute_dtype(model, dtype):
    """Activation / weight compute dtype for every module that creates activations
    from raw inputs (patch embeddings, the waveform front end)."""
    for m in model.modules():
        if hasattr(m, "compute_dtype"):
            m.compute_dtype = dtype
    return model


__all__ = ["set_compute_dtype", "torch"]

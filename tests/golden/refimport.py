"""Import the read-only reference (/root/reference) on CPU for golden-vector
generation.  Used ONLY by tests/golden/make_golden.py in the build container;
nothing on the GPU box imports it (the reference does not travel).

Recipe from SURVEY.md §8c: import transformers first, stub the modules the
reference imports but never uses on the forward/backward path (timm's
DropPath/trunc_normal_, mmengine, tensorflow, cv2, librosa, pydub, moviepy,
GPUtil), then inject the missing ``Mlp`` import into the VST module (Q1).
"""
import os
import sys
import types

REF = "/root/reference"


def _stub(name, **attrs):
    import importlib.machinery
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    import transformers  # noqa: F401  (must precede the librosa stub)
    from transformers import Wav2Vec2Config, Wav2Vec2Model  # noqa: F401  (resolve lazy imports first)
    import torch
    import torch.nn as nn

    class DropPath(nn.Module):
        """timm DropPath semantics: per-sample Bernoulli keep, scaled by 1/keep."""
        def __init__(self, drop_prob=0.0):
            super().__init__()
            self.drop_prob = drop_prob

        def forward(self, x):
            if self.drop_prob == 0.0 or not self.training:
                return x
            keep = 1 - self.drop_prob
            shape = (x.shape[0],) + (1,) * (x.ndim - 1)
            return x * x.new_empty(shape).bernoulli_(keep) / keep

    def to_2tuple(x):
        return tuple(x) if isinstance(x, (list, tuple)) else (x, x)

    timm = _stub("timm")
    timm.models = _stub("timm.models")
    timm.models.layers = _stub("timm.models.layers", DropPath=DropPath,
                               trunc_normal_=nn.init.trunc_normal_, to_2tuple=to_2tuple)
    _stub("mmengine", Config=object, DictAction=object)

    class _TFDummy:
        pass
    _stub("tensorflow", Tensor=_TFDummy, Variable=_TFDummy)
    _stub("cv2")
    _stub("librosa")
    _stub("pydub", AudioSegment=object)
    mp = _stub("moviepy")
    mp.editor = _stub("moviepy.editor")
    _stub("GPUtil", showUtilization=lambda *a, **k: None)

    if REF not in sys.path:
        sys.path.insert(0, REF)
    import src.utils as U
    import src.models.video_swin_transformer as VST
    VST.Mlp = U.Mlp  # Q1: video_swin_transformer.py:217 uses Mlp without importing it
    from src.models.ModalFusion import FusionModel
    from src.models.audioTransformer import Audio2D
    from src.models.swin_transformer2d import SwinTransformerV2
    S2 = sys.modules["src.models.swin_transformer2d"]
    return types.SimpleNamespace(U=U, VST=VST, FusionModel=FusionModel, Audio2D=Audio2D,
                                 SwinTransformerV2=SwinTransformerV2, S2=S2, torch=torch)

"""CPU: the MI355X InceptionVideoClassifier has exactly the reference's state_dict keys and
shapes (tests/golden/inception_keys.json, written by make_golden.py from /root/reference/src/models/IResNet.py)."""
import json
import os
import types

from fixtures import GOLDEN


def test_inception_state_dict_keys():
    from deepfake_amd.models.IResNet import InceptionVideoClassifier
    ref = json.load(open(os.path.join(GOLDEN, "inception_keys.json")))
    args = types.SimpleNamespace(bn_momentum=0.1, num_frames=2, classify_drop=0.0)
    m = InceptionVideoClassifier(args, num_classes=1, drop_rate=0.0)
    got = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert got == ref


def test_build_model_inception_slot():
    """--video_encoder inception builds the reference's current video branch (train.py:32) and fused model
    (train.py:42-46) with the reference's module tree."""
    import config
    from deepfake_amd.models.fused import build_model
    from deepfake_amd.models.IResNet import InceptionVideoClassifier
    a = config.get_opt(["--modality", "video", "--video_encoder", "inception", "--config", "c1", "--num_frames", "8"])
    m = build_model(a)
    assert isinstance(m, InceptionVideoClassifier) and m.drop_rate == a.swin_drop
    a = config.get_opt(["--modality", "fused", "--video_encoder", "inception", "--config", "c1", "--num_frames", "8"])
    m = build_model(a)
    assert isinstance(m.vExtract, InceptionVideoClassifier) and m.vExtract.use_feat
    assert m.video_projection.in_features == 1024

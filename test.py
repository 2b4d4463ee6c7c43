"""Inference / submission entry point — the reference's test.py:28-73 + src/submit.py (SubmitCtl):
build the model, optionally load --fused_ckpt_path (--Resume), run the test split and append
'video_name,probability' rows to prediction.csv, then write prediction_full.csv with a header (the
reference's test.py:58-61 refers to an undefined `result` there; here it is the returned dict).

    python test.py --modality fused --config c1 -b 2 --Resume --fused_ckpt_path ckpt.pth
"""
import json
import os
import sys
import threading

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from config import get_opt  # noqa: E402
from deepfake_amd.data import DeepFakeSet  # noqa: E402
from deepfake_amd.models.fused import CONFIGS, build_model  # noqa: E402
from deepfake_amd.submit import SubmitCtl  # noqa: E402
from deepfake_amd.utils import Logger, seed_torch  # noqa: E402


def test(args, logger, out_dir="."):
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    model = build_model(args, compute_dtype=dt)
    cfg = CONFIGS[args.config]
    data = DeepFakeSet(args, logger=logger, clip_shape=dict(T=cfg["T"], H=cfg["H"], W=cfg["W"], seconds=cfg["seconds"]))
    data.setup(threading.Event())
    device = torch.device("cuda:0")
    tester = SubmitCtl(model, args, device, data, logger)
    if args.Resume:
        tester.load_ckpt(args)
    result = tester.submit(os.path.join(out_dir, "prediction.csv"))
    with open(os.path.join(out_dir, "prediction_full.csv"), "w") as f:
        f.write("video_name,y_pred\n")
        for key, value in result.items():
            f.write("{0},{1}\n".format(key, value))
    return result


if __name__ == '__main__':
    opt = get_opt()
    logger = Logger(opt.log_dir)
    logger(json.dumps(opt.__dict__, indent=4))
    seed_torch(opt.random_seed)
    test(opt, logger)

"""Golden vectors for the f2 frame transform, generated with PIL 12.2 in the build container.

    python tests/golden/make_pil_fixtures.py      -> tests/golden/pil_frames.npz

The reference transforms every decoded frame as a PIL image (src/utils.py:32-33 Image.fromarray, then
data/data_process.py:55-69) and the mel JPEG (:162, Image.open(...).convert('RGB')) with the same transform.
torchvision is absent here, so this script makes the PIL calls torchvision's PIL path makes:
  T.Resize((h, w))       -> img.resize((w, h), Image.BILINEAR)
  T.Resize(224) (eval)   -> the shorter side to 224, the longer int(224 * long / short), then the same resize
  T.RandomHorizontalFlip -> img.transpose(Image.FLIP_LEFT_RIGHT); T.RandomVerticalFlip -> FLIP_TOP_BOTTOM
  T.RandomRotation(90)   -> img.rotate(angle, Image.NEAREST, expand=False, center=None, fillcolor=(0, 0, 0))
Inputs are regenerated from golden_cases.pil_test_image (seeded); the fixture holds the uint8 outputs (before
ToTensor / Normalize, which the tests apply in fp32) and the per-frame flips / angles."""
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_cases as GC  # noqa: E402

import torch  # noqa: E402


def train_transform(img, flip, angle, size=224):
    img = img.resize((size, size), Image.BILINEAR)
    if flip & 1:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
    if flip & 2:
        img = img.transpose(Image.FLIP_TOP_BOTTOM)
    return img.rotate(angle, Image.NEAREST, expand=False, center=None, fillcolor=(0, 0, 0))


def eval_size(h, w, short=224):
    return (int(short * h / w), short) if w <= h else (short, int(short * w / h))


def main():
    c = GC.PIL_FRAMES
    g = torch.Generator().manual_seed(c["seed"])
    out = {}
    # the reference's per-frame draw order: hflip, vflip, rotation angle
    def draw(n):
        fl, an = [], []
        for _ in range(n):
            hf = bool(torch.rand(1, generator=g) < 0.5)
            vf = bool(torch.rand(1, generator=g) < 0.5)
            an.append(float(torch.empty(1).uniform_(-90.0, 90.0, generator=g).item()))
            fl.append(int(hf) | (int(vf) << 1))
        return np.array(fl, dtype=np.int32), np.array(an, dtype=np.float64)

    cases = {  # name: (h, w, channels, frames, augment)
        "resize720": (720, 1280, 3, 2, False),
        "aug180": (180, 320, 3, 4, True),
        "aug720": (720, 1280, 3, 2, True),
        "mel224": (224, 224, 1, 3, True),
        "aug_up": (100, 150, 3, 2, True),
    }
    for ci, (name, (h, w, ch, n, aug)) in enumerate(cases.items()):
        fl, an = draw(n) if aug else (np.zeros(n, np.int32), np.zeros(n))
        base = c["seed"] * 1000 + 10 * ci          # frame i is pil_test_image(base + i, ...)
        res = []
        for i in range(n):
            arr = GC.pil_test_image(base + i, h, w, ch)
            img = Image.fromarray(arr).convert("RGB")
            res.append(np.asarray(train_transform(img, int(fl[i]), float(an[i])) if aug else
                                  img.resize((224, 224), Image.BILINEAR)))
        out[name] = np.stack(res)
        out[name + ":flips"], out[name + ":angles"] = fl, an
        out[name + ":seed"] = np.array(base)
    arr = GC.pil_test_image(c["seed"] * 1000 + 999, 720, 1280, 3)
    eh, ew = eval_size(720, 1280)
    out["eval720"] = np.asarray(Image.fromarray(arr).resize((ew, eh), Image.BILINEAR))[None]
    np.savez_compressed(os.path.join(HERE, c["name"] + ".npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()

"""Synthetic stand-in for the reference's media pipeline (data/data_process.py:17-234): the same
DeepFakeSet / DeepFake surface, item layout and collate functions, but clips are generated from a
seeded stream instead of decoded from mp4 files (no media ships with the repo; the benchmark metric
is defined on synthetic clips).

Items follow DeepFake.__getitem__ (:135-173) with modality 'fused':
  ({"Video": frames, "Audio": mel input, "PAudio": waveform (np.float32, raw)}, label, name)
  mel input: 'image' -> [3,224,224] fp32 (the normalised cached JPEG), 'uint8' -> [224,224] grey image (the
             trainer normalises it on the GPU), 'wave' -> 22.05 kHz waveform (the GPU builds the mel image,
             deepfake_amd.media, then normalises it)
  frames: 'normalized' -> [T,3,H,W] fp32, what extract_frames + T.Normalize produce (:55-69, utils.py:22-39)
          'uint8'      -> [T,H,W,3] uint8 decoded RGB frames; the trainer normalises them on the GPU
                          (deepfake_amd.kernels.frame_normalize: ToTensor + Normalize fused)
The test split yields (features, name) like the reference's test set.  Batches are collated by
fusion_collate / fusion_collate_test (src/utils.py:129-165): Video/Audio stacked, PAudio a list.
"""
import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _rng(seed, index):
    return np.random.Generator(np.random.Philox(key=(int(seed) << 32) + int(index)))


class DeepFake(Dataset):
    """Synthetic clips: label ~ Bernoulli(0.5); frames, mel image and waveform from the seeded stream."""

    def __init__(self, args, split="train", n=64, seed=0, frames="normalized", T=None, H=224, W=224, seconds=4,
                 mel_source="image"):
        self.args, self.split, self.n, self.seed = args, split, int(n), int(seed) + {"train": 0, "val": 1, "test": 2}[split]
        self.frames = frames
        self.mel_source = mel_source
        self.T = T or getattr(args, "num_frames", 32)
        self.H, self.W, self.seconds = H, W, seconds
        self.modality = getattr(args, "modality", "fused")
        self.test = split == "test"

    def __len__(self):
        return self.n

    def _video(self, g):
        u8 = g.integers(0, 256, size=(self.T, self.H, self.W, 3), dtype=np.uint8)
        if self.frames == "uint8":
            return torch.from_numpy(u8)
        x = torch.from_numpy(u8).permute(0, 3, 1, 2).float().div(255)          # T.ToTensor
        mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
        std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
        return x.sub(mean).div(std)                                               # T.Normalize

    def __getitem__(self, index):
        g = _rng(self.seed, index)
        name = f"synthetic_{self.split}_{index:06d}.mp4"
        label = torch.tensor(float(g.uniform() < 0.5), dtype=torch.float32)
        video = self._video(g)
        if self.mel_source == "uint8":       # the cached grey JPEG as decoded (data_process.py:83-93,162)
            mel = torch.from_numpy(g.integers(0, 256, size=(224, 224), dtype=np.uint8))
        elif self.mel_source == "wave":      # the waveform librosa.load hands generate_mel_spectrogram (22.05 kHz)
            mel = torch.from_numpy((0.1 * g.standard_normal(int(22050 * self.seconds))).astype(np.float32))
        else:
            mel = torch.from_numpy(g.standard_normal((3, 224, 224), dtype=np.float32))
        wave = (0.1 * g.standard_normal(int(16000 * self.seconds))).astype(np.float32)
        feat = {"video": video, "audio": mel, "paudio": wave.copy()}.get(self.modality)
        if self.modality == "fused":
            feat = {"Video": video, "Audio": mel, "PAudio": wave}
        if self.test:
            return feat, name
        return feat, label, name


def fusion_collate(batch):
    """src/utils.py:129-147."""
    features, labels, filenames = zip(*batch)
    out = {"Video": torch.stack([f["Video"] for f in features]), "Audio": torch.stack([f["Audio"] for f in features]),
           "PAudio": [f["PAudio"] for f in features]}
    return out, torch.stack(labels), filenames


def fusion_collate_test(batch):
    """src/utils.py:149-165."""
    features, filenames = zip(*batch)
    out = {"Video": torch.stack([f["Video"] for f in features]), "Audio": torch.stack([f["Audio"] for f in features]),
           "PAudio": [f["PAudio"] for f in features]}
    return out, filenames


def collate_opt(batch):
    """src/utils.py:122-127 (waveform modality: a list of variable-length arrays)."""
    features, labels, filenames = zip(*batch)
    return list(features), torch.stack(labels), filenames


class DeepFakeSet:
    """data/data_process.py:176-234: setup() then train/val/test dataloaders."""

    def __init__(self, args, world_size=None, rank=None, logger=None, clip_shape=None):
        self.args = args
        self.batch_size = args.batch_size
        self.num_workers = getattr(args, "num_workers", 0)
        self.world_size, self.rank, self.logger = world_size, rank, logger
        self.modality = getattr(args, "modality", "fused")
        self.clip_shape = clip_shape or {}
        self.trainset = self.valset = self.testset = None

    def setup(self, event=None, stage=None):
        a, kw = self.args, dict(frames=getattr(self.args, "frames", "normalized"),
                                mel_source=getattr(self.args, "mel_source", "image"), **self.clip_shape)
        seed = getattr(a, "random_seed", 0) * 7919 + (self.rank or 0)      # distinct clips per rank
        self.trainset = DeepFake(a, "train", getattr(a, "train_clips", 64), seed, **kw)
        self.valset = DeepFake(a, "val", getattr(a, "val_clips", 16), seed, **kw)
        self.testset = DeepFake(a, "test", getattr(a, "test_clips", 16), seed, **kw)

    def _loader(self, ds, shuffle, collate):
        return DataLoader(ds, batch_size=self.batch_size, shuffle=shuffle, num_workers=self.num_workers,
                          collate_fn=collate, drop_last=shuffle,
                          generator=torch.Generator().manual_seed(getattr(self.args, "random_seed", 0)))

    def _collate(self, test=False):
        if self.modality == "fused":
            return fusion_collate_test if test else fusion_collate
        return collate_opt if self.modality == "paudio" and not test else None

    def train_dataloader(self):
        return self._loader(self.trainset, True, self._collate())

    def val_dataloader(self):
        return self._loader(self.valset, False, self._collate())

    def test_dataloader(self):
        return self._loader(self.testset, False, self._collate(test=True))

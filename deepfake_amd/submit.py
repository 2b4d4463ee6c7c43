"""SubmitCtl — inference / submission controller of the reference (src/submit.py:23-120) on the HIP path:
the model in eval mode over the test split, probabilities appended to prediction.csv as
'video_name,probability' rows (src/submit.py:88,110), checkpoints in the reference's format
({'epoch', 'checkpoint': state_dict, 'optimizer'}) loaded with weights_only=True, strict=False, with the
'module.' prefix stripped for single-modality checkpoints (:50-74)."""
import torch

from .trainer import normalize_wave, pad_longest, prepare_video
from .utils import Logger


class SubmitCtl:
    def __init__(self, model, args, device, dataset, logger=None, processor=None):
        self.device = device
        self.batch_size = args.batch_size
        self.modality = args.modality
        self.logger = logger or Logger(None)
        self.log_step = args.log_step
        self.model_s = self.model = model.to(device)
        self.testloader = dataset.test_dataloader()

    def load_ckpt(self, args):
        path = args.fused_ckpt_path if self.modality == "fused" else (
            args.audio_ckpt_path if self.modality == "audio" else args.video_ckpt_path)
        sd = torch.load(path, map_location="cpu", weights_only=True)["checkpoint"]
        if self.modality != "fused":
            sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
        self.model_s.load_state_dict(sd, strict=False)
        self.logger(f"Load Finetuned Model From:{path}")

    def _features(self, feat):
        if self.modality == "fused":
            wave = normalize_wave(pad_longest(feat["PAudio"]).to(self.device))
            return (prepare_video(feat["Video"], self.device), feat["Audio"].to(self.device), wave)
        if self.modality == "paudio":
            return normalize_wave(pad_longest(feat).to(self.device))
        if self.modality == "video":
            return prepare_video(feat, self.device)
        return feat.to(self.device)

    def submit(self, path="prediction.csv"):
        res = {}
        self.model.eval()
        with torch.no_grad(), open(path, "a") as f:
            for iter_id, (feat, names) in enumerate(self.testloader):
                out = self.model(self._features(feat)).float().reshape(-1).cpu()
                for name, v in zip(names, out.numpy()):
                    f.write("{0},{1}\n".format(name, v))
                    res[name] = float(v)
                if iter_id % self.log_step == 0:
                    self.logger("|step {:4d} |total {:4d}| Rate% {:.3f}".format(
                        iter_id, len(self.testloader), iter_id / len(self.testloader) * 100))
        self.logger("Test Score Prediction Done")
        return res

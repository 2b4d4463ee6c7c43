"""Training entry point — the reference's train.py:29-75 on the MI355X build.

    python train.py --modality fused --config c2 -b 8 --accum_step 1 -e 1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...

Same flow: flags (config.py), Logger, seed_torch, model by --modality, DeepFakeSet(...).setup(event),
Trainer(model, args, device, data, logger, processor), optional --Resume, train() unless --skip_learning /
--val_model, eval on --val_model.  Differences, all deliberate:
  * one process per GPU (torchrun) with RCCL gradient all-reduce instead of DataParallel;
  * the fused model's video slot is the north-star SwinTransformer3D (the reference's train.py:45 builds
    InceptionVideoClassifier);
  * synthetic clips (deepfake_amd.data) — the reference's media files, and its pretrained weights
    (git-LFS pointers), are not available;
  * the wav2vec2 processor is the on-device normalisation (deepfake_amd.trainer.normalize_wave).
"""
import atexit
import json
import os
import signal
import sys
import threading

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from config import get_opt  # noqa: E402
from deepfake_amd.data import DeepFakeSet  # noqa: E402
from deepfake_amd.models.fused import CONFIGS, build_model  # noqa: E402
from deepfake_amd.trainer import Trainer  # noqa: E402
from deepfake_amd.utils import Logger, seed_torch  # noqa: E402


def handle_exit(*_):
    print('Program Killed by signal')


def shut_sub_prog(event: threading.Event):
    event.set()


def init_distributed():
    """torchrun environment -> one process per GPU (RCCL); plain launch -> single process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        # captured bucket all-reduces need RCCL work events outside torch's event cache (see bench.py)
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
        os.environ.setdefault("TORCH_FR_BUFFER_SIZE", "256")   # watchdog drain before capture (ddp.py)
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo",
                                device_id=torch.device("cuda", local) if torch.cuda.is_available() else None)
    rank = dist.get_rank() if dist.is_initialized() else 0
    return rank, world, torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")


def train(args, logger):
    rank, world, device = init_distributed()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    model = build_model(args, compute_dtype=dt)
    cfg = CONFIGS[args.config]
    event = threading.Event()
    atexit.register(shut_sub_prog, event)
    data = DeepFakeSet(args, world_size=world, rank=rank, logger=logger,
                       clip_shape=dict(T=cfg["T"], H=cfg["H"], W=cfg["W"], seconds=cfg["seconds"]))
    data.setup(event)
    trainer = Trainer(model, args, device, data, logger, processor=None, compute_dtype=dt, graph=args.graph)
    if args.Resume:
        trainer.load_ckpt(args)
    if not (args.skip_learning or args.val_model):
        trainer.train()
    if args.val_model:
        trainer.eval(data.val_dataloader(), 0, 0, 0)
    if dist.is_initialized():
        dist.destroy_process_group()
    return trainer


if __name__ == '__main__':
    opt = get_opt()
    logger = Logger(opt.log_dir)
    logger(f'processId: {os.getpid()}')
    logger(f'prarent processId: {os.getppid()}')
    logger(json.dumps(opt.__dict__, indent=4))
    atexit.register(handle_exit)
    signal.signal(signal.SIGTERM, handle_exit)
    signal.signal(signal.SIGINT, handle_exit)
    seed_torch(opt.random_seed)
    train(opt, logger)

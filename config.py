"""Command-line flags of the training / inference entry points — the reference's config.py:3-45
(every one of its 31 flags, same names, types and defaults) plus the MI355X build's own:

  --config {c1,c2,c4,c5}   model/clip shapes of BASELINE.json's configurations (deepfake_amd.models.fused)
  --dtype {bf16,fp32}      compute precision (fp32 = the parity mode of the 1e-3 logits gate)
  --graph / --no-graph     replay the whole training step as one HIP graph (default on)
  --train_clips / --val_clips / --test_clips   size of the synthetic split (no media ships with the repo)
  --frames {normalized,uint8}   synthetic frames as the reference's transform output (fp32, ImageNet
                           normalised) or as decoded uint8 RGB frames normalised on the GPU
  --bucket_mb              gradient all-reduce bucket size
  --deterministic          dropout / DropPath / SpecAugment / LayerDrop off (the parity setting, Q12)
  --video_encoder {swin,inception}   video slot: the north-star Video Swin 3D (default) or the reference's
                           current InceptionVideoClassifier (Inception-ResNet-v2 + NeXtVLAD, train.py:32,44)

Launch one process per GPU: python -m torch.distributed.run --nproc-per-node N train.py ...
"""
import argparse


def build_parser():
    parser = argparse.ArgumentParser(description="Deepfake")
    # DATA (config.py:6-11)
    parser.add_argument('--data_root', type=str, default=r'/data/lingfeng/full_data/phase1')
    parser.add_argument('--modality', type=str, default='audio')
    parser.add_argument('--num_frames', type=int, default=32, help='extract fixed number of frames')
    parser.add_argument('--force_generate', action='store_true', help='force process audio file')
    parser.add_argument('-nu', '--num_workers', type=int, default=1, help='thread number')
    # Model (config.py:13-28)
    parser.add_argument('--video_pretrained_dir', type=str,
                        default='checkpoints/swin_small_patch244_window877_kinetics400_1k.pth')
    parser.add_argument('--audio_pretrained_dir', type=str, default='checkpoints/swinv2_tiny_patch4_window16_256.pth')
    parser.add_argument('--classify_drop', type=float, default=0.1, help='MLP_dropout_rate')
    parser.add_argument('--swin_drop', type=float, default=0.1, help='VST_dropout_rate')
    parser.add_argument('--soft', type=float, default=0.01, help='NCE-SoftParam')
    parser.add_argument('--num_hiddens', type=int, default=128, help='Hidden Num of Classifier')
    parser.add_argument('--video_pool', type=str, help='VST Pool Method')
    parser.add_argument('--audio_ckpt_path', type=str, default=None)
    parser.add_argument('--video_ckpt_path', type=str, default=None)
    parser.add_argument('--paudio_ckpt_path', type=str, default=None)
    parser.add_argument('--fused_ckpt_path', type=str, default=None)
    parser.add_argument('--bn_momentum', type=float, default=0.1, help='BatchNorm Momentum')
    parser.add_argument('--Resume', action='store_true', help='resume model from ckpt')
    # Learning (config.py:30-41)
    parser.add_argument('--random_seed', type=int, default=42, help='torch random seed')
    parser.add_argument('-b', '--batch_size', type=int, default=8, help='input batch size for training (default: 32)')
    parser.add_argument('--accum_step', type=int, default=4, help='Gradient Accumulation Steps')
    parser.add_argument('-cuda', '--use_cuda', type=bool, default=True, help='Use cuda or not')
    parser.add_argument('--align_loss_rate', type=float, default=0.4, help='Ratio of Loss_align')
    parser.add_argument('--l2_decacy', type=float, default=0.05)
    parser.add_argument('-e', '--epochs', type=int, default=50, help='input training epoch for training (default: 50)')
    parser.add_argument('-lr', '--learning_rate', type=float, default=1e-4,
                        help='input learning rate for training (default: 1e-4)')
    parser.add_argument('--model_save', type=int, default=5, help='save model per %d round')
    parser.add_argument('--skip_learning', action='store_true', help='skip train stage and get submission')
    parser.add_argument('--val_model', action='store_true', help='Eval Model Performence on Eval Set')
    # Log (config.py:43-44)
    parser.add_argument('--log_step', type=int, default=10)
    parser.add_argument('--log_dir', type=str, default=None)
    # MI355X build
    parser.add_argument('--config', type=str, default='c2', choices=['c1', 'c2', 'c4', 'c5'])
    parser.add_argument('--dtype', type=str, default='bf16', choices=['bf16', 'fp32'])
    parser.add_argument('--graph', dest='graph', action='store_true', default=True)
    parser.add_argument('--no-graph', dest='graph', action='store_false')
    parser.add_argument('--train_clips', type=int, default=64)
    parser.add_argument('--val_clips', type=int, default=16)
    parser.add_argument('--test_clips', type=int, default=16)
    parser.add_argument('--frames', type=str, default='normalized', choices=['normalized', 'uint8'])
    # f2 media front end on the device: mel slot input as the reference's cached image (fp32 normalised or the
    # uint8 grey image) or as the raw 22.05 kHz waveform (device mel-spectrogram image); train-time frame
    # augmentation (flips, rotation) of uint8 frames on the device
    parser.add_argument('--mel_source', type=str, default='image', choices=['image', 'uint8', 'wave'])
    parser.add_argument('--augment', action='store_true')
    parser.add_argument('--bucket_dtype', type=str, default='fp32', choices=['fp32', 'bf16'])
    parser.add_argument('--bucket_mb', type=float, default=64.0)
    parser.add_argument('--deterministic', action='store_true')
    parser.add_argument('--video_encoder', type=str, default='swin', choices=['swin', 'inception'])
    return parser


def get_opt(argv=None):
    return build_parser().parse_args(argv)

"""Conv3D patch-embed forward (dfk_patch_embed_fwd) cold timing at C2 (B=8), as bench.py's roofline_conv3d.
Tuning knobs via env: DFK_PE_PERCU (workgroups per CU), DFK_PE_DEPTH (rows of clip loads in flight)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from deepfake_amd.models.fused import CONFIGS  # noqa: E402

r = bench.conv3d_roofline(CONFIGS["c2"], 8, 50)
print(os.environ.get("DFK_PE_PERCU", "-"), os.environ.get("DFK_PE_DEPTH", "-"), r["avg_launch_ms"], r["frac"], flush=True)

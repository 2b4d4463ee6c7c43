"""Generate golden vectors by running the REFERENCE modules on CPU (fp32).

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py
Writes tests/golden/*.npz.  Weights are never stored: every case re-creates
them with oracle.fill.named_fill_ (deterministic per state_dict key), and
inputs / upstream gradients come from oracle.fill.randn / synthetic_inputs
(seeded Philox streams), so the fixtures hold inputs only when tiny and always
the reference outputs.

Cases follow SURVEY.md §8c "Golden vectors to commit".
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from refimport import import_reference  # noqa: E402
from oracle.fill import named_fill_, randn, synthetic_inputs  # noqa: E402
import golden_cases as GC  # noqa: E402

R = import_reference()
torch = R.torch
torch.set_num_threads(8)
VST = R.VST


BIG = 65536  # larger tensors are stored as a strided sample + sum + norm (fixture_compress)


def save(name, _big=BIG, _sample=8192, **arrays):
    out = {}
    for k, v in arrays.items():
        a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        out.update(GC.fixture_compress(k, a, _big, _sample))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: " + ", ".join(f"{k}{tuple(v.shape)}" for k, v in out.items()))


def grads_of(module, prefix=""):
    return {("g:" + prefix + n): p.grad.clone() for n, p in module.named_parameters() if p.grad is not None}


# ---------------------------------------------------------------- VST pieces
def case_window_attention():
    for c in GC.WATTN_CASES:
        m = VST.WindowAttention3D(c["dim"], c["full_window"], c["heads"], qkv_bias=True)
        named_fill_(m, seed=c["seed"])
        x = randn(c["seed"] + 1, (c["B_"], c["N"], c["dim"])).requires_grad_(True)
        mask = None
        if c.get("mask_dhw"):
            D, H, W = c["mask_dhw"]
            mask = VST.compute_mask(D, H, W, tuple(c["full_window"]), tuple(c["shift"]), torch.device("cpu"))
        y = m(x, mask)
        gy = randn(c["seed"] + 2, y.shape)
        y.backward(gy)
        save(c["name"], y=y, dx=x.grad, **grads_of(m))


def _block(c):
    m = VST.SwinTransformerBlock3D(c["dim"], c["heads"], window_size=tuple(c["window"]),
                                   shift_size=tuple(c["shift"]), qkv_bias=True)
    named_fill_(m, seed=c["seed"])
    B, D, H, W = c["shape"]
    x = randn(c["seed"] + 1, (B, D, H, W, c["dim"])).requires_grad_(True)
    ws, ss = VST.get_window_size((D, H, W), tuple(c["window"]), tuple(c["shift"]))
    Dp = -(-D // ws[0]) * ws[0]
    Hp = -(-H // ws[1]) * ws[1]
    Wp = -(-W // ws[2]) * ws[2]
    mask = VST.compute_mask(Dp, Hp, Wp, ws, ss, torch.device("cpu"))
    y = m(x, mask)
    gy = randn(c["seed"] + 2, y.shape)
    y.backward(gy)
    save(c["name"], y=y, dx=x.grad, **grads_of(m))


def case_block():
    for c in GC.BLOCK_CASES:
        _block(c)


def case_block_c2():
    """C2 geometry: the stage-1 SW-MSA launch the bench's roofline reports (N=392, shift 4x3x3,
    a whole clip's 16x56x56 volume) and the stage-4 D-only shift (4,0,0) at 16x7x7."""
    _block(GC.BLOCK_C2_S1)
    _block(GC.BLOCK_C2_S4)


def case_block_c4():
    """C4 geometry (Swin-B video trunk): stage 1 (dim 128, 4 heads, N=392, shift 4x3x3) and stage 3 (dim 512,
    16 heads) — the blocks whose Linears the fp8 path runs on MX-fp8 GEMMs."""
    _block(GC.BLOCK_C4_S1)
    _block(GC.BLOCK_C4_S3)


def case_pretrained():
    """The reference's pretrained-weight loaders on synthetic checkpoints: SwinTransformer3D.inflate_weights
    (video_swin_transformer.py:566-632: 2-D -> 3-D patch-embed repeat / depth, bicubic RPB resize, repeat 2Wd-1) and
    the SwinV2 load_pretrained (src/utils.py:294-380).  Stores the loaded tensors (the randomly re-initialised rest
    is not comparable)."""
    import tempfile
    c = GC.PRETRAINED
    m = VST.SwinTransformer3D(**c["vst"])
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ck = GC.synth_swin2d_checkpoint(shapes, c["seed"])
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "swin2d.pth")
        torch.save(ck, path)
        m.pretrained = path
        m.inflate_weights(lambda *a: None)
    sd = m.state_dict()
    out = {"v:" + k: sd[k] for k in ck["model"] if k in sd and "relative_position_index" not in k}
    v2 = R.S2.SwinTransformerV2(**c["mel"])
    shapes2 = {k: tuple(t.shape) for k, t in v2.state_dict().items()}
    ck2 = GC.synth_swinv2_checkpoint(shapes2, c["seed"] + 1)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "swinv2.pth")
        torch.save(ck2, path)
        args = types.SimpleNamespace(audio_ckpt_path=path, audio_pretrained_dir=path)
        import src.utils as RU
        RU.load_pretrained(args, v2, lambda *a: None)
    sd2 = v2.state_dict()
    out.update({"a:" + k: sd2[k] for k in ck2["checkpoint"]})
    save(c["name"], _big=4096, _sample=1024, **out)


def case_mel_c2():
    """SwinV2-B mel stage-3 block pair (reference BasicLayer: W-MSA then SW-MSA shift 3)."""
    c = GC.MEL_C2_S3
    m = R.S2.BasicLayer(dim=c["dim"], input_resolution=c["res"], depth=2, num_heads=c["heads"],
                        window_size=c["window"], pretrained_window_size=c["pretrained"])
    named_fill_(m, seed=c["seed"])
    H, W = c["res"]
    x = randn(c["seed"] + 1, (c["B"], H * W, c["dim"])).requires_grad_(True)
    y = m(x)
    gy = randn(c["seed"] + 2, y.shape)
    y.backward(gy)
    save(c["name"], y=y, dx=x.grad, **grads_of(m))


def case_patch_embed_merge():
    c = GC.PATCH_EMBED
    m = VST.PatchEmbed3D(tuple(c["patch"]), 3, c["dim"], norm_layer=torch.nn.LayerNorm)
    named_fill_(m, seed=c["seed"])
    x = randn(c["seed"] + 1, c["shape"])
    y = m(x)
    gy = randn(c["seed"] + 2, y.shape)
    y.backward(gy)
    save(c["name"], y=y, **grads_of(m))
    for c in GC.MERGE_CASES:
        m = VST.PatchMerging(c["dim"])
        named_fill_(m, seed=c["seed"])
        x = randn(c["seed"] + 1, c["shape"]).requires_grad_(True)
        y = m(x)
        gy = randn(c["seed"] + 2, y.shape)
        y.backward(gy)
        save(c["name"], y=y, dx=x.grad, **grads_of(m))


def case_vst_c1():
    c = GC.VST_C1
    m = VST.SwinTransformer3D(**c["kwargs"])
    named_fill_(m, seed=c["seed"])
    m.eval()  # (Q2: returns None, do not chain)
    x = randn(c["seed"] + 1, c["shape"])
    with torch.no_grad():
        y = m(x)
    save(c["name"], y=y)


# ------------------------------------------------------------------ wav2vec2
def w2v_model(layers):
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    cfg = Wav2Vec2Config.from_json_file(GC.W2V_CONFIG_JSON)
    for k, v in GC.w2v_overrides(layers).items():
        setattr(cfg, k, v)
    cfg._attn_implementation = "eager"
    return Wav2Vec2Model(cfg)


def case_w2v():
    c = GC.W2V_C1
    m = w2v_model(c["layers"])
    named_fill_(m, seed=c["seed"])
    m.train()  # all stochastic pieces are disabled by w2v_overrides
    _, _, wave, _ = synthetic_inputs(c["B"], 2, 16, 16, c["seconds"], seed=c["seed"] + 1)
    out = m(wave)
    h = out.last_hidden_state
    gy = randn(c["seed"] + 2, h.shape)
    h.backward(gy)
    g = grads_of(m)
    keep = {k: v for k, v in g.items() if any(s in k for s in GC.W2V_GRAD_KEYS)}
    save(c["name"], y=h, extract=out.extract_features, **keep)


# -------------------------------------------------------------- fusion head
class _Ident(torch.nn.Module):
    def forward(self, x):
        return x


def case_head():
    c = GC.HEAD
    args = types.SimpleNamespace(soft=0.01, classify_drop=0.0, swin_drop=0.0)
    m = R.FusionModel(args, _Ident(), _Ident(), _Ident(), out_dim=1, video_dim=c["video_dim"],
                      audio_dim=c["audio_dim"], paudio_dim=768)
    named_fill_(m, seed=c["seed"])
    B = c["B"]
    fv = randn(c["seed"] + 1, (B, c["video_dim"])).requires_grad_(True)
    fa = randn(c["seed"] + 2, (B, c["audio_dim"])).requires_grad_(True)
    fp = randn(c["seed"] + 3, (B, 768)).requires_grad_(True)
    logits = {}
    m.classify.register_forward_hook(lambda mod, i, o: logits.__setitem__("z", o.detach().clone()))
    m.train()
    p = m((fv, fa, fp))
    gy = randn(c["seed"] + 4, p.shape)
    p.backward(gy)
    out = dict(p_train=p, z_train=logits["z"], dfv=fv.grad, dfa=fa.grad, dfp=fp.grad,
               rm=m.norm.running_mean, rv=m.norm.running_var, **grads_of(m))
    m.eval()
    with torch.no_grad():
        pe = m((fv, fa, fp))
    save(c["name"], p_eval=pe, z_eval=logits["z"], **out)


# ----------------------------------------------------------- fused C1 model
class VSTFeat(torch.nn.Module):
    """Build glue (Q8): [B,T,C,H,W] -> permute -> SwinTransformer3D -> mean(D,H,W)."""
    def __init__(self, vst):
        super().__init__()
        self.vst = vst

    def forward(self, x):
        return self.vst(x.permute(0, 2, 1, 3, 4)).mean(dim=[2, 3, 4])


def build_fused_ref(cfg):
    args = types.SimpleNamespace(soft=0.01, classify_drop=0.0, swin_drop=0.0)
    vst = VST.SwinTransformer3D(**cfg["vst"])
    mel = R.SwinTransformerV2(**cfg["mel"])
    w2v = w2v_model(cfg["w2v_layers"])
    pa = R.Audio2D(args, w2v, num_classes=1, use_feat=True)
    m = R.FusionModel(args, VSTFeat(vst), mel, pa, out_dim=1, video_dim=cfg["video_dim"],
                      audio_dim=cfg["audio_dim"], paudio_dim=768)
    return m


def case_fused_c1():
    c = GC.FUSED_C1
    m = build_fused_ref(c)
    named_fill_(m, seed=c["seed"])
    video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
    logits = {}
    m.classify.register_forward_hook(lambda mod, i, o: logits.__setitem__("z", o.detach().clone()))
    m.eval()
    with torch.no_grad():
        pe = m((video, mel, wave))
    z_eval = logits["z"]
    # one training step exactly as src/trainer.py:80-88,124-148,280-297 (accum_step=1)
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=c["lr"], momentum=0.9, weight_decay=c["wd"])
    opt.zero_grad()
    p = m((video, mel, wave))
    loss = torch.nn.BCELoss()(p, label)
    loss.backward()
    gnorm = {("gn:" + n): q.grad.norm() for n, q in m.named_parameters() if q.grad is not None}
    opt.step()
    psum = {("ps:" + n): q.detach().double().sum() for n, q in m.named_parameters()}
    save(c["name"], p_eval=pe, z_eval=z_eval, p_train=p, z_train=logits["z"], loss=loss, **gnorm, **psum)


def _sampled_err(a, ref, sample):
    """The parity tests' error metric (tests/fixtures.error) on the fixture's own sampling."""
    a, ref = a.double().reshape(-1), ref.double().reshape(-1)
    step = -(-ref.numel() // sample) if ref.numel() > sample else 1
    e = ((a[::step] - ref[::step]).abs().max() / ref[::step].abs().max().clamp_min(1e-12)).item()
    en = abs(a.norm().item() - ref.norm().item()) / max(ref.norm().item(), 1e-12)
    return max(e, en)


def _fused_train_grads(c, sample):
    """One training forward + BCE backward of the reference fused model (src/trainer.py:124-148,280-282);
    returns the per-parameter gradient tensors (compressed) and the step's outputs.

    The same step is also run under the reference's own bf16 autocast (torch.autocast(bfloat16) on CPU):
    ``ea:<param>`` is that run's gradient error against the fp32 one, in the parity tests' metric — the
    error bf16 arithmetic itself costs this model, which bounds what any bf16 implementation can meet."""
    m = build_fused_ref(c)
    named_fill_(m, seed=c["seed"])
    video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
    logits = {}
    m.classify.register_forward_hook(lambda mod, i, o: logits.__setitem__("z", o.detach().clone()))
    m.eval()
    with torch.no_grad():
        pe = m((video, mel, wave))
    z_eval = logits["z"]
    m.train()
    p = m((video, mel, wave))
    loss = torch.nn.BCELoss()(p, label)
    loss.backward()
    z_train = logits["z"]
    g = {("g:" + n): q.grad.clone() for n, q in m.named_parameters() if q.grad is not None}
    m2 = build_fused_ref(c)
    named_fill_(m2, seed=c["seed"])
    m2.train()
    m2.classify.register_forward_hook(lambda mod, i, o: logits.__setitem__("z", o.detach().clone()))
    with torch.autocast("cpu", dtype=torch.bfloat16):
        p2 = m2((video, mel, wave))
    torch.nn.BCELoss()(p2.float(), label).backward()
    ea = {("ea:" + n): _sampled_err(q.grad, g["g:" + n], sample)
          for n, q in m2.named_parameters() if q.grad is not None and ("g:" + n) in g}
    za = (logits["z"].double() - z_train.double()).abs().max() / z_train.double().abs().max()
    return m, dict(p_eval=pe, z_eval=z_eval, p_train=p, z_train=z_train, loss=loss, ea_logits=za, **g, **ea)


def case_fused_c1_grads():
    """The fused C1 train step's per-parameter gradient TENSORS (strided samples + norms)."""
    c = GC.FUSED_C1
    _, out = _fused_train_grads(c, GC.GRAD_SAMPLE_C1)
    save("fused_c1_grads", _big=GC.GRAD_SAMPLE_C1, _sample=GC.GRAD_SAMPLE_C1, **out)


def case_fused_c2():
    """The whole north-star model at C2 shapes (Swin-T 32x224x224, SwinV2-B mel, wav2vec2-base 4 s), B=2:
    eval logits/probabilities and one training forward+backward with every gradient tensor (sampled)."""
    c = GC.FUSED_C2
    _, out = _fused_train_grads(c, GC.GRAD_SAMPLE_C2)
    save(c["name"], _big=GC.GRAD_SAMPLE_C2, _sample=GC.GRAD_SAMPLE_C2, **out)


def case_fused_c2_fp8():
    """The anchor of C4's fp8 gradient bounds: the reference fused C2 model's training step in fp32 with its
    video stage-3/4 qkv / proj / fc1 / fc2 Linears on MX-fp8 operands emulated (tests/mx_ref.MXLinearFn: forward
    and input-gradient operands fake-quantised, weight gradients unquantised — what models.set_fp8 runs), against
    the same step unquantised.  ``ef8:<param>`` is that gradient error in the parity metric (tests/fixtures.error),
    z / loss the emulated run's logits and loss."""
    sys.path.insert(0, os.path.dirname(HERE))
    import mx_ref
    c = GC.FUSED_C2
    video, mel, wave, label = synthetic_inputs(c["B"], c["T"], c["H"], c["W"], c["seconds"], seed=c["seed"] + 1)
    grads, outs = [], []
    for emulate in (False, True):
        m = build_fused_ref(c)
        named_fill_(m, seed=c["seed"])
        if emulate:
            n = 0
            for li in (2, 3):
                for blk in m.vExtract.vst.layers[li].blocks:
                    for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
                        lin.forward = (lambda x, _l=lin: mx_ref.MXLinearFn.apply(x, _l.weight, _l.bias))
                        n += 1
            assert n == 32, n
        logits = {}
        m.classify.register_forward_hook(lambda mod, i, o: logits.__setitem__("z", o.detach().clone()))
        m.train()
        p = m((video, mel, wave))
        loss = torch.nn.BCELoss()(p, label)
        loss.backward()
        grads.append({n: q.grad.clone() for n, q in m.named_parameters() if q.grad is not None})
        outs.append((logits["z"], loss.detach()))
    g32, g8 = grads
    ef8 = {("ef8:" + n): _sampled_err(g8[n], g32[n], GC.GRAD_SAMPLE_C2) for n in g32 if n in g8}
    zf = (outs[1][0].double() - outs[0][0].double()).abs().max() / outs[0][0].double().abs().max()
    # relative L2 of all gradients together, over the tensors the parity test weighs (the analytically-zero
    # ones excluded as tests/test_gpu_c2.GRAD_FLOOR does)
    top = max(float(g.double().norm()) for g in g32.values())
    num = den = 0.0
    for n in g32:
        if n in g8 and float(g32[n].double().norm()) >= 1e-6 * top:
            num += float(((g8[n].double() - g32[n].double()) ** 2).sum())
            den += float((g32[n].double() ** 2).sum())
    l2 = (num / den) ** 0.5
    print("ef8 median", sorted(ef8.values())[len(ef8) // 2], "max", max(ef8.values()), "logits", float(zf), "l2", l2)
    save("fused_c2_fp8", z_train8=outs[1][0], loss8=outs[1][1], ef8_logits=zf, ef8_l2=l2, **ef8)


def case_state_keys():
    """state_dict keys + shapes of the reference fused model at C1 and C2 (371 keys at C1)."""
    import json
    out = {}
    for c in (GC.FUSED_C1, GC.FUSED_C2):
        sd = build_fused_ref(c).state_dict()
        out[c["name"]] = [[k, list(v.shape)] for k, v in sd.items()]
    with open(os.path.join(HERE, "state_keys.json"), "w") as f:
        json.dump(out, f)
    print("state_keys:", {k: len(v) for k, v in out.items()})


def case_config_flags():
    """Every flag of the reference's config.py:3-45 (dest, option strings, type, default, action) from
    its own argparse parser, for the entry-surface test of config.py."""
    import argparse
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("ref_config", os.path.join("/root/reference", "config.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    captured = {}
    orig = argparse.ArgumentParser.parse_args

    def grab(self, args=None, namespace=None):
        captured["parser"] = self
        return orig(self, [], namespace)
    argparse.ArgumentParser.parse_args = grab
    try:
        mod.get_opt()
    finally:
        argparse.ArgumentParser.parse_args = orig
    flags = []
    for a in captured["parser"]._actions:
        if a.dest == "help":
            continue
        flags.append(dict(dest=a.dest, options=list(a.option_strings), type=getattr(a.type, "__name__", None),
                          default=a.default, action=type(a).__name__))
    with open(os.path.join(HERE, "config_flags.json"), "w") as f:
        json.dump(flags, f, indent=1)
    print("config flags:", len(flags))


def case_inception():
    """the reference's InceptionVideoClassifier (IResNet.py:331-393 over InceptionResV2.py) at a
    small frame size (B=2 clips x T=2 frames x 75x75 — the smallest input the stem/reductions accept), training
    mode (batch-statistics BatchNorm), drop_rate 0 and classify_drop 0 (the reference's F.dropout calls are
    always on, so dropout is off for a deterministic fixture): probabilities, BCE loss, gradients (sampled),
    BatchNorm running statistics after the step, the eval-mode probabilities that follow, and the state_dict
    keys / shapes."""
    import json
    import src.models.IResNet as IR
    c = GC.INCEPTION
    args = types.SimpleNamespace(bn_momentum=0.1, num_frames=c["T"], classify_drop=0.0)
    m = IR.InceptionVideoClassifier(args, num_classes=1, drop_rate=0.0)
    named_fill_(m, seed=c["seed"])
    x = randn(c["seed"] + 1, (c["B"], c["T"], 3, c["HW"], c["HW"]))
    label = torch.tensor([1.0, 0.0])
    m.train()
    prob = m(x)
    loss = torch.nn.BCELoss()(prob, label)
    loss.backward()
    out = dict(prob=prob.detach(), loss=loss.detach())   # x is re-drawn by oracle.fill.randn(seed + 1, shape)
    out.update({k: v for k, v in grads_of(m).items()})
    sd = m.state_dict()
    for k in c["bn_keys"]:
        out["s:" + k] = sd[k]
    m.eval()
    with torch.no_grad():
        out["prob_eval"] = m(x)
    save(c["name"], _big=c["sample"], _sample=c["sample"], **out)
    with open(os.path.join(HERE, "inception_keys.json"), "w") as f:
        json.dump([[k, list(v.shape)] for k, v in sd.items()], f)


if __name__ == "__main__":
    only = sys.argv[1:]
    for fn in [case_window_attention, case_block, case_patch_embed_merge, case_vst_c1, case_w2v, case_head,
               case_fused_c1, case_block_c2, case_mel_c2, case_fused_c1_grads, case_fused_c2, case_state_keys,
               case_config_flags, case_inception, case_block_c4, case_pretrained, case_fused_c2_fp8]:
        if not only or fn.__name__ in only:
            fn()

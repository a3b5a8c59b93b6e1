"""K-UNet (stabilityai/sd-x2-latent-upscaler architecture, models/kunet.py)
against an independent NCHW re-statement of k-diffusion's image_v1 denoiser
(ResConvBlock / AdaGN / SelfAttention2d / CrossAttention2d / binomial
Down/Upsample2d, UNet skip order) written here from the published model
description, fed the same weights by key.  fp32 on CPU.

Checkpoint parity is unpinned: the published diffusers checkpoint is not
available offline (models/kunet.py docstring)."""
import math

import torch
import torch.nn.functional as F

from chiaswarm_amd.models.kunet import TINY_X2_K, KUNet2DConditionModel
from chiaswarm_amd.models.layers import init_random_
from chiaswarm_amd.schedulers import get_scheduler


def _lin(sd, p, x):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


def _adagn(sd, p, x, emb, groups):
    w, b = _lin(sd, p + ".linear", emb).chunk(2, dim=-1)
    return F.group_norm(x, groups, eps=1e-5) * (w[:, :, None, None] + 1) + b[:, :, None, None]


def _conv(sd, p, x, pad):
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), padding=pad)


def _resconv(sd, p, x, emb, gs):
    cin = x.shape[1]
    cmid = sd[p + ".conv1.weight"].shape[0]
    h = F.gelu(_adagn(sd, p + ".norm1", x, emb, max(1, cin // gs)))
    h = _conv(sd, p + ".conv1", h, 1)
    h = F.gelu(_adagn(sd, p + ".norm2", h, emb, max(1, cmid // gs)))
    h = _conv(sd, p + ".conv2", h, 1)
    skip = _conv(sd, p + ".conv_shortcut", x, 0) if p + ".conv_shortcut.weight" in sd else x
    return h + skip


def _heads_attn(q, k, v, nh):
    b, sq, c = q.shape
    d = c // nh
    q, k, v = (t.reshape(b, -1, nh, d).transpose(1, 2) for t in (q, k, v))
    att = (q @ k.transpose(-1, -2) / math.sqrt(d)).softmax(-1)
    return (att @ v).transpose(1, 2).reshape(b, sq, c)


def _kattn(sd, p, x, emb, ctx, gs, head):
    n, c, h, w = x.shape
    nh = max(1, c // head)
    g = max(1, c // gs)
    if p + ".attn1.to_q.weight" in sd:
        hn = _adagn(sd, p + ".norm1", x, emb, g).flatten(2).transpose(1, 2)
        o = _heads_attn(_lin(sd, p + ".attn1.to_q", hn), _lin(sd, p + ".attn1.to_k", hn),
                        _lin(sd, p + ".attn1.to_v", hn), nh)
        x = x + _lin(sd, p + ".attn1.to_out.0", o).transpose(1, 2).reshape(n, c, h, w)
    hn = _adagn(sd, p + ".norm2", x, emb, g).flatten(2).transpose(1, 2)
    cn = F.layer_norm(ctx, (ctx.shape[-1],), sd[p + ".attn2.norm_cross.weight"], sd[p + ".attn2.norm_cross.bias"])
    o = _heads_attn(_lin(sd, p + ".attn2.to_q", hn), _lin(sd, p + ".attn2.to_k", cn), _lin(sd, p + ".attn2.to_v", cn),
                    nh)
    return x + _lin(sd, p + ".attn2.to_out.0", o).transpose(1, 2).reshape(n, c, h, w)


def _kernel(c, scale):
    k1 = torch.tensor([1.0, 3.0, 3.0, 1.0]) / 8 * scale
    k = k1[:, None] * k1[None, :]
    wt = torch.zeros(c, c, 4, 4)
    wt[range(c), range(c)] = k
    return wt


def _down(x):
    return F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), _kernel(x.shape[1], 1.0), stride=2)


def _up(x):
    return F.conv_transpose2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), _kernel(x.shape[1], 2.0), stride=2, padding=3)


def reference_forward(sd, cfg, x, c_noise, cond, ctx):
    """k-diffusion image_v1 semantics on NCHW tensors."""
    f = 2 * math.pi * c_noise[:, None] * sd["time_proj.weight"][None]
    temb = torch.cat([f.cos(), f.sin()], -1) + F.linear(cond, sd["time_embedding.cond_proj.weight"])
    emb = F.gelu(_lin(sd, "time_embedding.linear_2", F.gelu(_lin(sd, "time_embedding.linear_1", temb))))
    gs, head = cfg.group_size, cfg.attention_head_dim
    h = _conv(sd, "conv_in", x, 0)
    skips = []
    n = len(cfg.block_out_channels)
    for i in range(n):
        if i > 0:  # k-diffusion: a DBlock downsamples at its start
            h = _down(h)
        for j in range(cfg.layers_per_block[i]):
            h = _resconv(sd, f"down_blocks.{i}.resnets.{j}", h, emb, gs)
            if cfg.cross_attn[i]:
                h = _kattn(sd, f"down_blocks.{i}.attentions.{j}", h, emb, ctx, gs, head)
        skips.append(h)
    for k, i in enumerate(reversed(range(n))):
        skip = skips.pop()
        if k > 0:
            h = torch.cat([h, skip], 1)
        for j in range(cfg.layers_per_block[i]):
            h = _resconv(sd, f"up_blocks.{k}.resnets.{j}", h, emb, gs)
            if cfg.cross_attn[i]:
                h = _kattn(sd, f"up_blocks.{k}.attentions.{j}", h, emb, ctx, gs, head)
        if i > 0:  # ... and a UBlock upsamples at its end
            h = _up(h)
    return _conv(sd, "conv_out", h, 0)


@torch.no_grad()
def test_kunet_matches_kdiffusion_reference():
    torch.manual_seed(0)
    cfg = TINY_X2_K
    m = KUNet2DConditionModel(cfg).eval()
    init_random_(m, seed=3)
    # random (not unit) norms / biases / Fourier weights so every term matters
    g = torch.Generator().manual_seed(5)
    for name, p in m.named_parameters():
        if p.dim() == 1:
            p.copy_(torch.randn(p.shape, generator=g) * (0.5 if "bias" in name else 1.0)
                    + (1.0 if name.endswith("norm_cross.weight") else 0.0))
    sd = {k: v.float() for k, v in m.state_dict().items()}
    b, hw = 2, 8
    x = torch.randn(b, cfg.in_channels, hw, hw)
    c_noise = torch.log(torch.tensor([2.5, 0.3])) / 4
    cond = torch.randn(b, cfg.time_cond_proj_dim)
    ctx = torch.randn(b, 7, cfg.cross_attention_dim)
    ref = reference_forward(sd, cfg, x, c_noise, cond, ctx)
    out = m(x.permute(0, 2, 3, 1).contiguous(), c_noise, cond, cross_kv=m.encode_context(ctx), drop_variance=False)
    out = out.permute(0, 3, 1, 2)
    assert out.shape == (b, cfg.out_channels, hw, hw)
    err = (out - ref).abs().max() / ref.abs().max()
    assert err < 1e-4, float(err)
    # variance channel dropped on the default path: same first 4 channels
    out4 = m(x.permute(0, 2, 3, 1).contiguous(), c_noise, cond, cross_kv=m.encode_context(ctx))
    assert out4.shape[-1] == 4
    assert torch.allclose(out4.permute(0, 3, 1, 2), ref[:, :4], atol=1e-4 * float(ref.abs().max()))


def test_kunet_state_dict_layout():
    m = KUNet2DConditionModel(TINY_X2_K)
    keys = set(m.state_dict())
    # diffusers K-block naming
    for k in ("time_proj.weight", "time_embedding.cond_proj.weight", "time_embedding.linear_1.weight",
              "down_blocks.0.resnets.0.norm1.linear.weight", "down_blocks.1.attentions.0.attn2.norm_cross.weight",
              "down_blocks.2.attentions.0.attn1.to_q.weight", "up_blocks.0.attentions.0.norm1.linear.weight",
              "up_blocks.1.resnets.0.conv_shortcut.weight", "conv_in.weight", "conv_out.bias"):
        assert k in keys, k
    assert "time_embedding.cond_proj.bias" not in keys
    assert not any(k.startswith("up_blocks.2.attentions") for k in keys)  # top level: no attention
    assert not any("conv_shortcut.bias" in k for k in keys)


def test_k_denoiser_euler_is_karras_preconditioned():
    """x0 = x / (s^2 + 1) + s / sqrt(s^2 + 1) * F; one Euler step to sigma_next."""
    s = get_scheduler("EulerDiscreteScheduler", use_karras_sigmas=False, prediction_type="k_denoiser")
    s.set_timesteps(4)
    x = torch.randn(1, 4, 4, 4)
    fo = torch.randn(1, 4, 4, 4)
    sig, nxt = float(s.sigmas[0]), float(s.sigmas[1])
    x0 = x / (sig ** 2 + 1) + sig / math.sqrt(sig ** 2 + 1) * fo
    want = x0 + (x - x0) / sig * nxt
    got = s.step(fo, x)
    assert torch.allclose(got, want, atol=1e-5)

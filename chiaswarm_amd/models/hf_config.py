"""Model construction from a checkpoint's own configuration files — the
``from_pretrained`` half of the reference's model loading:

* ``pipeline_type.from_pretrained(model_name, revision=...)`` builds every
  component from ``model_index.json`` + ``<component>/config.json``
  (swarm/diffusion/diffusion_func.py:41-46, swarm/video/tx2vid.py:24-30,
  swarm/audio/audioldm.py:19-20);
* ``scheduler_type.from_config(pipeline.scheduler.config, use_karras_sigmas=True)``
  carries the checkpoint's training schedule, prediction type, steps offset
  and timestep spacing into whichever sampler the hive names
  (swarm/diffusion/diffusion_func.py:72-74).

Here the same files are parsed into this package's config dataclasses
(``UNetConfig``, ``VAEConfig``, ``CLIPTextConfig``) and scheduler kwargs.  Any
option the modules here do not implement raises ``UnsupportedConfig`` (a
``ValueError``: the job comes back fatal with the option named) instead of
silently building a different network.  Name heuristics remain only for
directories without config files (random-init runs, old hand-made stores).
"""
from __future__ import annotations

import dataclasses
import json
import os

from .clip import CLIPTextConfig
from .xlmr import is_xlmr_config, xlmr_text_config
from .unet import UNetConfig
from .vae import VAEConfig


class UnsupportedConfig(ValueError):
    pass


def read_json(path: str) -> dict | None:
    try:
        with open(path) as f:
            return json.load(f)
    except FileNotFoundError:
        return None


def component_config(weights_dir: str | None, sub: str, name: str = "config.json") -> dict | None:
    if not weights_dir:
        return None
    return read_json(os.path.join(weights_dir, sub, name) if sub else os.path.join(weights_dir, name))


def _expect(cfg: dict, key: str, allowed, what: str):
    v = cfg.get(key)
    if v is not None and v not in allowed:
        raise UnsupportedConfig(f"{what}: {key}={v!r} is not supported (supported: {sorted(map(str, allowed))})")


_DOWN = {"CrossAttnDownBlock2D", "DownBlock2D"}
_UP = {"CrossAttnUpBlock2D", "UpBlock2D"}


def unet_config(cfg: dict, what: str = "unet") -> UNetConfig:
    """diffusers ``UNet2DConditionModel`` config.json -> ``UNetConfig``."""
    for key, allowed in (("time_embedding_type", {"positional"}), ("resnet_time_scale_shift", {"default"}),
                         ("mid_block_type", {"UNetMidBlock2DCrossAttn"}), ("conv_in_kernel", {3}),
                         ("conv_out_kernel", {3}), ("attention_type", {"default"}), ("act_fn", {"silu"}),
                         ("encoder_hid_dim_type", {None}), ("addition_embed_type", {None, "text_time"}),
                         ("class_embed_type", {None, "timestep", "simple_projection", "projection"}),
                         ("flip_sin_to_cos", {True}), ("freq_shift", {0})):
        _expect(cfg, key, allowed, what)
    for key in ("dual_cross_attention", "only_cross_attention", "resnet_skip_time_act", "mid_block_only_cross_attention"):
        if cfg.get(key):
            raise UnsupportedConfig(f"{what}: {key}=True is not supported")
    for key in ("encoder_hid_dim", "time_cond_proj_dim", "time_embedding_dim", "timestep_post_act",
                "class_embeddings_concat_dim", "reverse_transformer_layers_per_block", "cross_attention_norm"):
        if cfg.get(key) is not None:
            raise UnsupportedConfig(f"{what}: {key}={cfg[key]!r} is not supported")
    for key, allowed in (("center_input_sample", {False}), ("downsample_padding", {1}),
                         ("mid_block_scale_factor", {1, 1.0}), ("resnet_out_scale_factor", {1, 1.0})):
        _expect(cfg, key, allowed, what)
    downs, ups = list(cfg.get("down_block_types", [])), list(cfg.get("up_block_types", []))
    bad = [b for b in downs if b not in _DOWN] + [b for b in ups if b not in _UP]
    if bad:
        raise UnsupportedConfig(f"{what}: block types {bad} are not supported")
    ch = tuple(cfg["block_out_channels"])
    lpb = cfg.get("layers_per_block", 2)
    if isinstance(lpb, (list, tuple)):
        if len(set(lpb)) != 1:
            raise UnsupportedConfig(f"{what}: per-block layers_per_block {lpb} is not supported")
        lpb = lpb[0]
    # diffusers' naming quirk: ``attention_head_dim`` holds the number of heads
    # unless ``num_attention_heads`` is given (UNet2DConditionModel.__init__)
    heads = cfg.get("num_attention_heads") or cfg.get("attention_head_dim", 8)
    heads = tuple(heads) if isinstance(heads, (list, tuple)) else heads
    tl = cfg.get("transformer_layers_per_block", 1)
    tl = tuple(tl) if isinstance(tl, (list, tuple)) else tl
    xd = cfg.get("cross_attention_dim", 1280)
    xd = tuple(xd) if isinstance(xd, (list, tuple)) else xd
    return UNetConfig(
        in_channels=cfg.get("in_channels", 4), out_channels=cfg.get("out_channels", 4), block_out_channels=ch,
        layers_per_block=int(lpb), down_block_types=tuple(downs), up_block_types=tuple(ups), num_heads=heads,
        cross_attention_dim=xd, use_linear_projection=bool(cfg.get("use_linear_projection", False)),
        transformer_layers_per_block=tl, norm_num_groups=cfg.get("norm_num_groups", 32),
        norm_eps=cfg.get("norm_eps", 1e-5), addition_embed_type=cfg.get("addition_embed_type"),
        addition_time_embed_dim=cfg.get("addition_time_embed_dim") or 256,
        projection_class_embeddings_input_dim=cfg.get("projection_class_embeddings_input_dim") or 2816,
        sample_size=cfg.get("sample_size") or 64, num_class_embeds=cfg.get("num_class_embeds"),
        class_embed_type=cfg.get("class_embed_type"),
        class_embeddings_concat=bool(cfg.get("class_embeddings_concat", False)))


def vae_config(cfg: dict, what: str = "vae") -> VAEConfig:
    """diffusers ``AutoencoderKL`` config.json -> ``VAEConfig``."""
    bad = [b for b in cfg.get("down_block_types", []) if b != "DownEncoderBlock2D"] + \
          [b for b in cfg.get("up_block_types", []) if b != "UpDecoderBlock2D"]
    if bad:
        raise UnsupportedConfig(f"{what}: block types {bad} are not supported")
    _expect(cfg, "act_fn", {"silu"}, what)
    if cfg.get("use_quant_conv") is False or cfg.get("use_post_quant_conv") is False:
        raise UnsupportedConfig(f"{what}: VAEs without quant convs are not supported")
    if cfg.get("mid_block_add_attention") is False:
        raise UnsupportedConfig(f"{what}: mid_block_add_attention=False is not supported")
    sf = cfg.get("scaling_factor")
    return VAEConfig(in_channels=cfg.get("in_channels", 3), out_channels=cfg.get("out_channels", 3),
                     latent_channels=cfg.get("latent_channels", 4),
                     block_out_channels=tuple(cfg.get("block_out_channels", (128, 256, 512, 512))),
                     layers_per_block=cfg.get("layers_per_block", 2), norm_num_groups=cfg.get("norm_num_groups", 32),
                     scaling_factor=float(sf) if sf is not None else 0.18215)


def clip_text_config(cfg: dict, what: str = "text_encoder") -> CLIPTextConfig:
    """transformers ``CLIPTextModel`` / ``CLIPTextModelWithProjection``
    config.json -> ``CLIPTextConfig``."""
    if "text_config" in cfg and "hidden_size" not in cfg:  # a full CLIPModel config: its text tower
        cfg = dict(cfg["text_config"])
    act = cfg.get("hidden_act", "quick_gelu")
    if act not in ("quick_gelu", "gelu"):
        raise UnsupportedConfig(f"{what}: hidden_act={act!r} is not supported")
    archs = cfg.get("architectures") or []
    vocab = cfg.get("vocab_size", 49408)
    eos = cfg.get("eos_token_id", vocab - 1)
    if eos == 2:  # legacy configs: transformers pools at argmax(input_ids) = the highest id, <|endoftext|>
        eos = vocab - 1
    return CLIPTextConfig(vocab_size=vocab, hidden_size=cfg.get("hidden_size", 512),
                          intermediate_size=cfg.get("intermediate_size", 2048),
                          num_layers=cfg.get("num_hidden_layers", 12), num_heads=cfg.get("num_attention_heads", 8),
                          max_position=cfg.get("max_position_embeddings", 77), act=act,
                          projection_dim=(cfg.get("projection_dim") or 768)
                          if "CLIPTextModelWithProjection" in archs else None,
                          eos_token_id=eos)


# scheduler_config.json keys this package's samplers understand (Scheduler.__init__
# and subclasses); everything else (solver_type, algorithm_type variants, ...) is
# checked by the sampler itself
SCHED_KEYS = ("num_train_timesteps", "beta_start", "beta_end", "beta_schedule", "prediction_type", "steps_offset",
              "timestep_spacing", "clip_sample", "clip_sample_range", "thresholding", "dynamic_thresholding_ratio",
              "sample_max_value", "set_alpha_to_one", "trained_betas")


def scheduler_kwargs(cfg: dict | None) -> dict:
    """The checkpoint scheduler's training-schedule fields, to build the sampler
    the hive names ``from_config`` (the reference: DPMSolverMultistepScheduler
    etc. ``.from_config(pipeline.scheduler.config, use_karras_sigmas=True)``)."""
    if not cfg:
        return {}
    out = {k: cfg[k] for k in SCHED_KEYS if k in cfg and cfg[k] is not None}
    if out.get("beta_schedule") not in (None, "scaled_linear", "linear", "squaredcos_cap_v2"):
        raise UnsupportedConfig(f"scheduler: beta_schedule={out['beta_schedule']!r} is not supported")
    if out.get("trained_betas") is not None:
        raise UnsupportedConfig("scheduler: trained_betas is not supported")
    if out.get("prediction_type") not in (None, "epsilon", "v_prediction", "sample"):
        raise UnsupportedConfig(f"scheduler: prediction_type={out['prediction_type']!r} is not supported")
    return out


@dataclasses.dataclass
class PipelineSpec:
    """What a diffusers pipeline directory declares: its class and component
    configs (parsed), plus the raw scheduler config for ``from_config``."""
    class_name: str
    unet: UNetConfig
    vae: VAEConfig
    text: list
    scheduler: dict
    components: dict
    tokenizer_pad: list  # per tokenizer: the pad token string (None: not declared)
    text_names: tuple = ("text_encoder",)  # component directory of each text encoder
    requires_aesthetics_score: bool = False  # SDXL refiner: aesthetic score in the time ids
    force_zeros_for_empty_prompt: bool = False  # SDXL: no negative prompt -> zero negative embeddings


def pipeline_spec(weights_dir: str) -> PipelineSpec | None:
    """Parse ``model_index.json`` and the component configs of an SD-family
    diffusers directory; None when the directory carries no ``model_index.json``
    (then the caller falls back to name heuristics)."""
    idx = read_json(os.path.join(weights_dir, "model_index.json"))
    if idx is None:
        return None
    comps = {k: v for k, v in idx.items() if not k.startswith("_") and isinstance(v, (list, tuple)) and v[0]}
    for need in ("unet", "vae"):
        if need not in comps:
            raise UnsupportedConfig(f"{weights_dir}: model_index.json has no {need!r} component")
    if "text_encoder" not in comps and "text_encoder_2" not in comps and "image_encoder" not in comps:
        # (StableDiffusionImageVariationPipeline conditions on a CLIP image encoder instead)
        raise UnsupportedConfig(f"{weights_dir}: model_index.json has no 'text_encoder' component")
    ucfg = component_config(weights_dir, "unet")
    vcfg = component_config(weights_dir, "vae")
    if ucfg is None or vcfg is None:
        raise UnsupportedConfig(f"{weights_dir}: unet/config.json or vae/config.json is missing")
    if ucfg.get("_class_name", "UNet2DConditionModel") != "UNet2DConditionModel":
        raise UnsupportedConfig(f"unet: {ucfg['_class_name']} is not a UNet2DConditionModel")
    text = []
    pads = []
    names = []
    for i, sub in enumerate(("text_encoder", "text_encoder_2")):
        if sub not in comps:
            continue
        tc = component_config(weights_dir, sub)
        if tc is None:
            raise UnsupportedConfig(f"{weights_dir}: {sub}/config.json is missing")
        cls = (comps[sub][1] if len(comps[sub]) > 1 else "") or ""
        if cls == "RobertaSeriesModelWithTransformation" or (not cls.startswith("CLIPTextModel")
                                                             and is_xlmr_config(tc)):
            # AltDiffusion: XLM-RoBERTa + transformation (models/xlmr.py)
            text.append(xlmr_text_config(tc, sub))
            names.append(sub)
            pads.append("<pad>")
            continue
        if cls and not cls.startswith("CLIPTextModel"):
            raise UnsupportedConfig(f"{sub}: {cls} is not supported (CLIPTextModel[WithProjection] / "
                                    "RobertaSeriesModelWithTransformation only)")
        if cls == "CLIPTextModelWithProjection":
            tc = dict(tc)
            tc.setdefault("architectures", [cls])
            if cls not in tc["architectures"]:
                tc["architectures"] = list(tc["architectures"]) + [cls]
        text.append(clip_text_config(tc, sub))
        names.append(sub)
        tok = "tokenizer" if i == 0 else "tokenizer_2"
        sp = component_config(weights_dir, tok, "special_tokens_map.json") or {}
        tk = component_config(weights_dir, tok, "tokenizer_config.json") or {}
        pad = sp.get("pad_token", tk.get("pad_token"))
        pads.append(pad.get("content") if isinstance(pad, dict) else pad)
    sched = component_config(weights_dir, "scheduler", "scheduler_config.json") or {}
    cls = idx.get("_class_name", "DiffusionPipeline")
    # diffusers' StableDiffusionXL*Pipeline constructors default this to True
    fz = bool(idx.get("force_zeros_for_empty_prompt", str(cls).startswith("StableDiffusionXL")))
    return PipelineSpec(cls, unet_config(ucfg), vae_config(vcfg), text, sched, comps, pads, tuple(names),
                        bool(idx.get("requires_aesthetics_score", False)), fz)


def controlnet_config(cfg: dict, what: str = "controlnet") -> tuple[UNetConfig, dict]:
    """diffusers ``ControlNetModel`` config.json -> (UNetConfig of its encoder
    copy, ControlNetModel keyword args)."""
    if cfg.get("_class_name", "ControlNetModel") != "ControlNetModel":
        raise UnsupportedConfig(f"{what}: {cfg['_class_name']} is not supported (ControlNetModel only)")
    _expect(cfg, "controlnet_conditioning_channel_order", {"rgb", "bgr"}, what)
    u = unet_config(cfg, what)
    kw = dict(cond_channels=tuple(cfg.get("conditioning_embedding_out_channels") or (16, 32, 96, 256)),
              cond_in=int(cfg.get("conditioning_channels") or 3),
              bgr=cfg.get("controlnet_conditioning_channel_order", "rgb") == "bgr",
              global_pool=bool(cfg.get("global_pool_conditions", False)))
    return u, kw


def unet3d_config(cfg: dict, what: str = "unet") -> UNetConfig:
    """diffusers ``UNet3DConditionModel`` config.json (ModelScope text-to-video)
    -> ``UNetConfig``.  Here ``attention_head_dim`` IS the head width (the 3D
    blocks build ``out_channels // attention_head_dim`` heads)."""
    if cfg.get("_class_name", "UNet3DConditionModel") != "UNet3DConditionModel":
        raise UnsupportedConfig(f"{what}: {cfg['_class_name']} is not a UNet3DConditionModel")
    flat = dict(cfg)
    flat["down_block_types"] = [b.replace("3D", "2D") for b in cfg.get("down_block_types", [])]
    flat["up_block_types"] = [b.replace("3D", "2D") for b in cfg.get("up_block_types", [])]
    ch = list(cfg["block_out_channels"])
    hd = cfg.get("attention_head_dim", 64)
    hds = list(hd) if isinstance(hd, (list, tuple)) else [hd] * len(ch)
    if any(c % h for c, h in zip(ch, hds)):
        raise UnsupportedConfig(f"{what}: channels {ch} not divisible by head dims {hds}")
    flat["num_attention_heads"] = [c // h for c, h in zip(ch, hds)]
    u = unet_config(flat, what)
    return dataclasses.replace(u, down_block_types=tuple(cfg["down_block_types"]),
                               up_block_types=tuple(cfg["up_block_types"]))


def clap_text_config(cfg: dict, what: str = "text_encoder"):
    """transformers ``ClapTextModelWithProjection`` config.json -> ``ClapTextConfig``."""
    from .clap import ClapTextConfig

    if "text_config" in cfg and "hidden_size" not in cfg:
        cfg = dict(cfg["text_config"], projection_dim=cfg.get("projection_dim", 512))
    act = cfg.get("hidden_act", "gelu")
    if act != "gelu":
        raise UnsupportedConfig(f"{what}: hidden_act={act!r} is not supported")
    pa = cfg.get("projection_hidden_act", "relu")
    if pa != "relu":
        raise UnsupportedConfig(f"{what}: projection_hidden_act={pa!r} is not supported")
    return ClapTextConfig(vocab=cfg.get("vocab_size", 50265), dim=cfg.get("hidden_size", 768),
                          depth=cfg.get("num_hidden_layers", 12), heads=cfg.get("num_attention_heads", 12),
                          mlp=cfg.get("intermediate_size", 3072), max_pos=cfg.get("max_position_embeddings", 514),
                          pad_id=cfg.get("pad_token_id", 1), eps=cfg.get("layer_norm_eps", 1e-12),
                          projection_dim=cfg.get("projection_dim", 512))


def hifigan_config(cfg: dict, what: str = "vocoder"):
    """transformers ``SpeechT5HifiGan`` config.json -> ``HifiGanConfig``."""
    from .vocoder import HifiGanConfig

    if cfg.get("leaky_relu_slope", 0.1) != 0.1:
        raise UnsupportedConfig(f"{what}: leaky_relu_slope={cfg['leaky_relu_slope']} is not supported")
    return HifiGanConfig(model_in_dim=cfg.get("model_in_dim", 64), sampling_rate=cfg.get("sampling_rate", 16000),
                         upsample_initial_channel=cfg.get("upsample_initial_channel", 512),
                         upsample_rates=tuple(cfg.get("upsample_rates", (4, 4, 4, 4))),
                         upsample_kernel_sizes=tuple(cfg.get("upsample_kernel_sizes", (8, 8, 8, 8))),
                         resblock_kernel_sizes=tuple(cfg.get("resblock_kernel_sizes", (3, 7, 11))),
                         resblock_dilation_sizes=tuple(tuple(d) for d in cfg.get(
                             "resblock_dilation_sizes", ((1, 3, 5), (1, 3, 5), (1, 3, 5)))),
                         normalize_before=bool(cfg.get("normalize_before", True)))

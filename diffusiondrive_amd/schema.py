"""State-dict key schema of the reference ``V2TransfuserModel`` (inference-relevant and not).

The drop-in boundary loads the reference's checkpoint layout unchanged (SURVEY.md §8b,
"Weights"): keys as ``V2TransfuserModel.state_dict()`` names them (the agent wrapper adds
the ``_transfuser_model.`` prefix, transfuser_agent.py:55,94-106). This module enumerates
those keys and shapes from the config alone, in the reference's registration order:

* timm ResNet trunks        transfuser_backbone.py:24-33,50-55 (timm resnet.py names)
* GPT fusion blocks         transfuser_backbone.py:279-431
* 1x1 channel adapters      transfuser_backbone.py:76-93
* FPN top-down              transfuser_backbone.py:144-151
* BEV / status / queries    transfuser_model_v2.py:38-45
* semantic head, tf decoder transfuser_model_v2.py:47-82
* agent head                transfuser_model_v2.py:83-87,165-205
* trajectory head           transfuser_model_v2.py:428-478, 297-341, 208-231, 259-269
* bev_proj                  transfuser_model_v2.py:96
"""
from collections import OrderedDict
from typing import List, Tuple

from .config import TransfuserConfig, trunk_blocks, trunk_channels

Entry = Tuple[str, Tuple[int, ...], str]  # (key, shape, kind)


def _bn(out, p, c):
    out += [(f"{p}.weight", (c,), "bn_w"), (f"{p}.bias", (c,), "bn_b"),
            (f"{p}.running_mean", (c,), "bn_mean"), (f"{p}.running_var", (c,), "bn_var"),
            (f"{p}.num_batches_tracked", (), "count")]


def _conv(out, p, cout, cin, k, bias=False):
    out.append((f"{p}.weight", (cout, cin, k, k), "conv"))
    if bias:
        out.append((f"{p}.bias", (cout,), "bias"))


def _linear(out, p, nout, nin, bias=True):
    out.append((f"{p}.weight", (nout, nin), "linear"))
    if bias:
        out.append((f"{p}.bias", (nout,), "bias"))


def _ln(out, p, c):
    out += [(f"{p}.weight", (c,), "ln_w"), (f"{p}.bias", (c,), "ln_b")]


def _mha(out, p, d):
    out += [(f"{p}.in_proj_weight", (3 * d, d), "linear"), (f"{p}.in_proj_bias", (3 * d,), "bias")]
    _linear(out, f"{p}.out_proj", d, d)


def _trunk(out, p, arch, in_chans):
    kind, layers = trunk_blocks(arch)
    _conv(out, f"{p}.conv1", 64, in_chans, 7)
    _bn(out, f"{p}.bn1", 64)
    exp = 1 if kind == "basic" else 4
    inplanes = 64
    for i, (planes, n) in enumerate(zip([64, 128, 256, 512], layers)):
        stride = 1 if i == 0 else 2
        for b in range(n):
            q = f"{p}.layer{i + 1}.{b}"
            if kind == "basic":
                _conv(out, f"{q}.conv1", planes, inplanes, 3)
                _bn(out, f"{q}.bn1", planes)
                _conv(out, f"{q}.conv2", planes, planes, 3)
                _bn(out, f"{q}.bn2", planes)
            else:
                _conv(out, f"{q}.conv1", planes, inplanes, 1)
                _bn(out, f"{q}.bn1", planes)
                _conv(out, f"{q}.conv2", planes, planes, 3)
                _bn(out, f"{q}.bn2", planes)
                _conv(out, f"{q}.conv3", planes * 4, planes, 1)
                _bn(out, f"{q}.bn3", planes * 4)
            if b == 0 and (stride != 1 or inplanes != planes * exp):
                _conv(out, f"{q}.downsample.0", planes * exp, inplanes, 1)
                _bn(out, f"{q}.downsample.1", planes * exp)
            inplanes = planes * exp


def state_dict_schema(cfg: TransfuserConfig) -> List[Entry]:
    out: List[Entry] = []
    img_ch = trunk_channels(cfg.image_architecture)
    lid_ch = trunk_channels(cfg.lidar_architecture)
    d, ffn = cfg.tf_d_model, cfg.tf_d_ffn
    _trunk(out, "_backbone.image_encoder", cfg.image_architecture, 3)
    _trunk(out, "_backbone.lidar_encoder", cfg.lidar_architecture, cfg.lidar_in_channels)
    ntok = (cfg.img_vert_anchors * cfg.img_horz_anchors
            + cfg.lidar_vert_anchors * cfg.lidar_horz_anchors)
    for i in range(4):
        c = img_ch[1 + i]
        p = f"_backbone.transformers.{i}"
        out.append((f"{p}.pos_emb", (1, ntok, c), "pos_emb"))
        for b in range(cfg.n_layer):
            q = f"{p}.blocks.{b}"
            _ln(out, f"{q}.ln1", c)
            _ln(out, f"{q}.ln2", c)
            for nm in ("key", "query", "value", "proj"):
                _linear(out, f"{q}.attn.{nm}", c, c)
            _linear(out, f"{q}.mlp.0", cfg.block_exp * c, c)
            _linear(out, f"{q}.mlp.2", c, cfg.block_exp * c)
        _ln(out, f"{p}.ln_f", c)
    for i in range(4):
        _conv(out, f"_backbone.lidar_channel_to_img.{i}", img_ch[1 + i], lid_ch[1 + i], 1, bias=True)
    for i in range(4):
        _conv(out, f"_backbone.img_channel_to_lidar.{i}", lid_ch[1 + i], img_ch[1 + i], 1, bias=True)
    bc = cfg.bev_features_channels
    _conv(out, "_backbone.up_conv5", bc, bc, 3, bias=True)
    _conv(out, "_backbone.up_conv4", bc, bc, 3, bias=True)
    _conv(out, "_backbone.c5_conv", bc, lid_ch[4], 1, bias=True)

    out.append(("_keyval_embedding.weight", (8 ** 2 + 1, d), "embedding"))
    out.append(("_query_embedding.weight", (1 + cfg.num_bounding_boxes, d), "embedding"))
    _conv(out, "_bev_downscale", d, 512, 1, bias=True)
    _linear(out, "_status_encoding", d, 8)
    _conv(out, "_bev_semantic_head.0", bc, bc, 3, bias=True)
    _conv(out, "_bev_semantic_head.2", cfg.num_bev_classes, bc, 1, bias=True)
    for i in range(cfg.tf_num_layers):
        p = f"_tf_decoder.layers.{i}"
        _mha(out, f"{p}.self_attn", d)
        _mha(out, f"{p}.multihead_attn", d)
        _linear(out, f"{p}.linear1", ffn, d)
        _linear(out, f"{p}.linear2", d, ffn)
        for n in (1, 2, 3):
            _ln(out, f"{p}.norm{n}", d)
    _linear(out, "_agent_head._mlp_states.0", ffn, d)
    _linear(out, "_agent_head._mlp_states.2", 5, ffn)
    _linear(out, "_agent_head._mlp_label.0", 1, d)

    npose = cfg.trajectory_sampling.num_poses
    p = "_trajectory_head"
    out.append((f"{p}.plan_anchor", (cfg.num_modes, npose, 2), "anchor"))
    _linear(out, f"{p}.plan_anchor_encoder.0", d, 512)
    _ln(out, f"{p}.plan_anchor_encoder.2", d)
    _linear(out, f"{p}.plan_anchor_encoder.3", d, d)
    _linear(out, f"{p}.time_mlp.1", 4 * d, d)
    _linear(out, f"{p}.time_mlp.3", d, 4 * d)
    for i in range(cfg.num_diff_layers):
        q = f"{p}.diff_decoder.layers.{i}"
        _linear(out, f"{q}.cross_bev_attention.attention_weights", npose, d)
        _linear(out, f"{q}.cross_bev_attention.output_proj", d, d)
        _conv(out, f"{q}.cross_bev_attention.value_proj.0", 256, 256, 3, bias=True)
        _mha(out, f"{q}.cross_agent_attention", d)
        _mha(out, f"{q}.cross_ego_attention", d)
        _linear(out, f"{q}.ffn.0", ffn, d)
        _linear(out, f"{q}.ffn.2", d, ffn)
        for n in (1, 2, 3):
            _ln(out, f"{q}.norm{n}", d)
        _linear(out, f"{q}.time_modulation.scale_shift_mlp.1", 2 * d, 256)
        t = f"{q}.task_decoder"
        _linear(out, f"{t}.plan_cls_branch.0", d, d)
        _ln(out, f"{t}.plan_cls_branch.2", d)
        _linear(out, f"{t}.plan_cls_branch.3", d, d)
        _ln(out, f"{t}.plan_cls_branch.5", d)
        _linear(out, f"{t}.plan_cls_branch.6", 1, d)
        _linear(out, f"{t}.plan_reg_branch.0", d, d)
        _linear(out, f"{t}.plan_reg_branch.2", d, d)
        _linear(out, f"{t}.plan_reg_branch.4", npose * 3, d)
    _linear(out, "bev_proj.0", d, 320)
    _ln(out, "bev_proj.2", d)
    return out


def schema_dict(cfg: TransfuserConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    return OrderedDict((k, s) for k, s, _ in state_dict_schema(cfg))

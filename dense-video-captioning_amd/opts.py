"""Command-line / YAML options (reference: opts.py:7-221).

Same flag names, types and defaults as the reference parser, so `cfgs/*.yml` files load unchanged; YAML keys
override flags, and `base_cfg_path` chains are followed recursively (base first), as in opts.py:214-221.
`parse_opts(argv)` additionally accepts an explicit argv list and a `cfg_root` for resolving the relative
cfg paths the reference's YAML files use.
"""
import argparse
import os

import numpy as np
import yaml

# (flag, type, default, extra-kwargs) -- grouped as in the reference parser
_FLAGS = [
    # run
    ("cfg_path", str, None, {}), ("id", str, "", {}), ("gpu_id", str, [], {"nargs": "+"}),
    ("seed", int, 777, {}), ("disable_cudnn", int, 0, {}),
    ("device", str, "cuda", {"choices": ["cpu", "cuda"]}),
    # data paths
    ("train_caption_file", str, "data/anet/captiondata/train_modified.json", {}),
    ("invalid_video_json", str, [], {"nargs": "+"}), ("val_caption_file", str, "data/anet/captiondata/val_1.json", {}),
    ("visual_feature_folder", str, "data/anet/resnet_bn", {}),
    ("gt_file_for_auc", str, "data/anet/captiondata/val_all.json", {"nargs": "+"}),
    ("gt_file_for_eval", str, ["data/anet/captiondata/val_1.json", "data/anet/captiondata/val_2.json"], {"nargs": "+"}),
    ("gt_file_for_para_eval", str, ["data/anet/captiondata/para/anet_entities_val_1_para.json",
                                    "data/anet/captiondata/para/anet_entities_val_2_para.json"], {"nargs": "+"}),
    ("dict_file", str, "data/anet/vocabulary_activitynet.json", {}),
    ("criteria_for_best_ckpt", str, "dvc", {"choices": ["dvc", "pc"]}),
    ("visual_feature_type", str, "c3d", {"choices": ["c3d", "resnet_bn", "resnet"]}),
    ("feature_dim", int, 500, {}), ("start_from", str, "", {}),
    ("start_from_mode", str, "last", {"choices": ["best", "last"]}),
    ("pretrain", str, None, {"choices": ["full", "encoder", "decoder"]}), ("pretrain_path", str, "", {}),
    # data loader
    ("nthreads", int, 4, {}), ("data_norm", int, 0, {}), ("data_rescale", int, 1, {}),
    ("feature_sample_rate", int, 1, {}), ("train_proposal_sample_num", int, 24, {}),
    ("gt_proposal_sample_num", int, 10, {}),
    # caption decoder
    ("vocab_size", int, 5747, {}),
    ("wordRNN_input_feats_type", str, "C", {"choices": ["C", "E", "C+E"]}),
    ("caption_decoder_type", str, "light", {"choices": ["none", "light", "standard"]}),
    ("rnn_size", int, 512, {}), ("num_layers", int, 1, {}), ("input_encoding_size", int, 512, {}),
    ("att_hid_size", int, 512, {}), ("drop_prob", float, 0.5, {}), ("max_caption_len", int, 30, {}),
    # transformer
    ("hidden_dim", int, 512, {}), ("num_queries", int, 100, {}), ("hidden_dropout_prob", float, 0.5, {}),
    ("layer_norm_eps", float, 1e-12, {}), ("caption_cost_type", str, "loss", {}),
    ("set_cost_caption", float, 0, {}), ("set_cost_class", float, 1, {}), ("set_cost_bbox", float, 5, {}),
    ("set_cost_giou", float, 2, {}), ("cost_alpha", float, 0.25, {}), ("cost_gamma", float, 2, {}),
    ("bbox_loss_coef", float, 5, {}), ("giou_loss_coef", float, 2, {}), ("count_loss_coef", float, 0, {}),
    ("caption_loss_coef", float, 0, {}), ("eos_coef", float, 0.1, {}), ("num_classes", int, 1, {}),
    ("dec_layers", int, 6, {}), ("enc_layers", int, 6, {}), ("transformer_ff_dim", int, 2048, {}),
    ("transformer_dropout_prob", float, 0.1, {}), ("frame_embedding_num", int, 100, {}),
    ("sample_method", str, "nearest", {"choices": ["nearest", "linear"]}), ("fix_xcw", int, 0, {}),
    # optimiser
    ("training_scheme", str, "all", {"choices": ["cap_head_only", "no_cap_head", "all"]}),
    ("epoch", int, 30, {}), ("batch_size", int, 1, {}), ("batch_size_for_eval", int, 1, {}),
    ("grad_clip", float, 100.0, {}), ("optimizer_type", str, "adam", {}), ("weight_decay", float, 0, {}),
    ("lr", float, 1e-4, {}), ("learning_rate_decay_start", float, 8, {}),
    ("learning_rate_decay_every", float, 3, {}), ("learning_rate_decay_rate", float, 0.5, {}),
    # saving / logging
    ("min_epoch_when_save", int, -1, {}), ("save_checkpoint_every", int, 1, {}), ("save_dir", str, "save", {}),
    # deformable DETR
    ("lr_backbone_names", str, ["None"], {"nargs": "+"}), ("lr_backbone", float, 2e-5, {}),
    ("lr_proj", int, 0, {}), ("lr_linear_proj_names", str, ["reference_points", "sampling_offsets"], {"nargs": "+"}),
    ("lr_linear_proj_mult", float, 0.1, {}),
    ("transformer_input_type", str, "queries", {"choices": ["gt_proposals", "learnt_proposals", "queries"]}),
    ("backbone", str, None, {}), ("position_embedding", str, "sine", {"choices": ("sine", "learned")}),
    ("position_embedding_scale", float, 2 * np.pi, {}), ("num_feature_levels", int, 4, {}),
    ("nheads", int, 8, {}), ("dec_n_points", int, 4, {}), ("enc_n_points", int, 4, {}),
    ("share_caption_head", int, 1, {}), ("cap_nheads", int, 8, {}), ("cap_dec_n_points", int, 4, {}),
    ("cap_num_feature_levels", int, 4, {}),
    # loss
    ("cls_loss_coef", float, 2, {}), ("focal_alpha", float, 0.25, {}), ("focal_gamma", float, 2.0, {}),
    # event counter
    ("max_eseq_length", int, 10, {}), ("lloss_gau_mask", int, 1, {}), ("lloss_beta", float, 1, {}),
    # scheduled sampling
    ("scheduled_sampling_start", int, -1, {}), ("basic_ss_prob", float, 0, {}),
    ("scheduled_sampling_increase_every", int, 2, {}), ("scheduled_sampling_increase_prob", float, 0.05, {}),
    ("scheduled_sampling_max_prob", float, 0.25, {}),
    # reranking
    ("ec_alpha", float, 0.3, {}),
]
_SWITCHES = ["disable_tqdm", "random_seed", "debug", "save_all_checkpoint", "with_box_refine", "dilation",
             "disable_mid_caption_heads"]


def make_parser():
    p = argparse.ArgumentParser()
    for name, typ, default, kw in _FLAGS:
        kw = dict(kw)
        if name == "cfg_path":
            kw["required"] = True
        p.add_argument("--" + name, type=typ, default=default, **kw)
    for name in _SWITCHES:
        p.add_argument("--" + name, action="store_true")
    p.add_argument("--no_aux_loss", dest="aux_loss", action="store_false")
    return p


def import_cfg(cfg_path, args, cfg_root=None):
    """Merge a YAML file (and its base_cfg_path chain, base first) into the dict `args`."""
    path = cfg_path if (cfg_root is None or os.path.isabs(cfg_path)) else os.path.join(cfg_root, cfg_path)
    with open(path, "r") as f:
        yml = yaml.safe_load(f) or {}
    if "base_cfg_path" in yml:
        import_cfg(yml["base_cfg_path"], args, cfg_root)
    args.update(yml)


def parse_opts(argv=None, cfg_root=None, **overrides):
    args = make_parser().parse_args(argv)
    if args.cfg_path:
        import_cfg(args.cfg_path, vars(args), cfg_root)
    if args.caption_decoder_type == "none":
        assert args.caption_loss_coef == 0
        assert args.set_cost_caption == 0
    for k, v in overrides.items():
        setattr(args, k, v)
    return args

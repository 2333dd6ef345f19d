"""Regenerate include/s3od_hip.h from the extern "C" definitions in s3od_amd/csrc/*.hip.

Each declaration carries the reference interface it replaces (REF below, file:line under
/root/reference or tf: = transformers' modeling_dinov3_vit.py).  s3od_amd/_lib.py parses the
header to build its ctypes bindings, so header, library and Python cannot drift apart.
"""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
REF = {
    "s3od_last_error": "error channel for every entry point (new; the reference raises Python exceptions)",
    "s3od_abi_version": "ABI version of this header",
    "s3od_linear_fwd": "nn.Linear / 1x1 nn.Conv2d forward: tf:modeling_dinov3_vit.py:294-357 (o_proj, up/down_proj), src/s3od/model.py:135-142 (projects), :185-191",
    "s3od_linear_dgrad": "autograd of nn.Linear w.r.t. input (reference: implicit torch autograd)",
    "s3od_linear_wgrad": "autograd of nn.Linear w.r.t. weight (reference: implicit torch autograd)",
    "s3od_qkv_rope_fwd": "DINOv3ViTAttention q/k/v_proj + apply_rotary_pos_emb: tf:modeling_dinov3_vit.py:294-314, 238-268",
    "s3od_conv_fwd": "nn.Conv2d forward (3x3 s1/s2, 1x1) + BatchNorm/ReLU/residual: src/s3od/model.py:144-159, 244-345, 437-452",
    "s3od_conv_dgrad": "nn.ConvTranspose2d forward (src/s3od/model.py:146-153, 437-439) and Conv2d input-gradient",
    "s3od_conv_wgrad": "Conv2d / ConvTranspose2d weight gradient (reference: implicit torch autograd)",
    "s3od_mask_heads_fwd": "MultiMaskHead.mask_heads (NM = 3 dinob / 1 dinol x Conv3x3+ReLU+Conv1x1) + torch.cat: src/s3od/model.py:440-467",
    "s3od_attn_fwd": "SDPA softmax(qk^T/8)v: tf:integrations/sdpa_attention.py:79-166 via tf:modeling_dinov3_vit.py:316-329",
    "s3od_patch_im2col": "DINOv3ViTEmbeddings.patch_embeddings Conv2d(3,768,16,16) im2col: tf:modeling_dinov3_vit.py:75-86",
    "s3od_token_prefix": "cat([cls, register_tokens, patches]): tf:modeling_dinov3_vit.py:88-92",
    "s3od_rope_table": "DINOv3ViTRopePositionEmbedding.forward: tf:modeling_dinov3_vit.py:96-200",
    "s3od_layernorm_fwd": "nn.LayerNorm(D = 768 | 1024, eps=1e-5) norm1/norm2: tf:modeling_dinov3_vit.py:419-445",
    "s3od_layernorm_bwd": "LayerNorm backward (reference: implicit torch autograd)",
    "s3od_cast_tap": "hidden_states[2,5,8,11] (dinob) / [4,11,17,23] (dinol) [:, 1+4:] taps: src/s3od/model.py:62-86, MT/model.py:28-32",
    "s3od_colsum": "bias gradients (reference: implicit torch autograd)",
    "s3od_colsum_ws": "workspace query of s3od_colsum: bytes of the caller-owned partial-sum buffer (new; torch autograd reduces internally)",
    "s3od_layerscale_bwd": "DINOv3ViTLayerScale backward: tf:modeling_dinov3_vit.py:337-343",
    "s3od_qkv_unrope": "apply_rotary_pos_emb backward: tf:modeling_dinov3_vit.py:238-268",
    "s3od_repack_weight": "weight layout for the kernels (the reference's state_dict layout is kept for params)",
    "s3od_repack_multi": "all kernel-layout weight repacks of one optimizer step in one launch (reference: none; PyTorch reads its fp32 parameters directly)",
    "s3od_bn_fold": "nn.BatchNorm2d eval-mode affine: src/s3od/model.py:326-343",
    "s3od_bn_finalize": "nn.BatchNorm2d train-mode batch statistics + running-stat update (momentum 0.1)",
    "s3od_affine_act": "BatchNorm apply + ReLU + residual: src/s3od/model.py:334-345, 383-393",
    "s3od_bn_bwd": "BatchNorm2d train-mode backward (reference: implicit torch autograd)",
    "s3od_bn_relu_bwd": "BatchNorm2d + ReLU train-mode backward with the ReLU mask recomputed from z (reference: implicit torch autograd of src/s3od/model.py:334-345)",
    "s3od_bilinear_fwd": "F.interpolate(bilinear, align_corners=False): src/s3od/model.py:395-403",
    "s3od_bilinear_bwd": "F.interpolate backward (reference: implicit torch autograd)",
    "s3od_avgpool": "classifier_head AdaptiveAvgPool2d(1): src/s3od/model.py:185-191",
    "s3od_iou_head_fwd": "classifier_head Linear-ReLU-Linear: src/s3od/model.py:185-191",
    "s3od_iou_head_bwd": "classifier_head backward (reference: implicit torch autograd)",
    "s3od_mask_heads_bwd": "MultiMaskHead.mask_heads backward prologue (reference: implicit torch autograd)",
    "s3od_mask_loss_fwd": "MaskLossHandler.compute_multi_mask_losses + aux MSE: synth_sod/.../model_training/loss.py:155-275",
    "s3od_mask_loss_bwd": "gradient of the multi-mask loss w.r.t. pred_masks / pred_iou logits: loss.py:190-275",
    "s3od_attn_bwd": "SDPA backward (reference: implicit torch autograd)",
    "s3od_attn_bwd_qkv": "SDPA backward + apply_rotary_pos_emb backward + q/k/v_proj output gradient in one pass (reference: implicit torch autograd of tf:modeling_dinov3_vit.py:238-268, 294-329)",
    "s3od_adamw_step": "torch.optim.AdamW(wd=0.05, betas=(0.9,0.999), eps=1e-8), 2 param groups: lightning_module.py:183-193",
    "s3od_sigmoid_unpad_resize": "remove_background post-processing: src/s3od/predictor.py:113-132, src/s3od/utils.py:32-37",
    "s3od_augment_sample": "get_transforms geometry (LongestMaxSize + PadIfNeeded + flip/affine/perspective/optical distortion) + Normalize, one launch per sample: synth_sod/src/synth_sod/model_training/transforms.py:12-64, 205-222",
    "s3od_augment_synthetic": "get_transforms(mode='synthetic') photometric OneOf groups on the geometric result: synth_sod/src/synth_sod/model_training/transforms.py:65-204, 220",
    "s3od_elastic_field": "ElasticTransform(alpha=1, sigma=25) displacement fields (albumentations 2.0.8 generate_displacement_fields): synth_sod/src/synth_sod/model_training/transforms.py:169-173",
    "s3od_augment_ws_floats": "workspace size of s3od_augment_synthetic (new; albumentations allocates numpy temporaries)",
    "s3od_eval_metrics": "EvaluationMetrics.step (MAE, MaxF/AvgF, S-measure) + EMeasure + WeightedFMeasure on device: synth_sod/src/synth_sod/model_training/metrics.py:14-424",
    "s3od_eval_metrics_ws": "scratch size of s3od_eval_metrics (new; the reference allocates numpy temporaries)",
    "s3od_preprocess": "BackgroundRemoval._preprocess normalisation: src/s3od/predictor.py:79-94",
    "s3od_linear_wgrad_ws": "workspace query of s3od_linear_wgrad: bytes of the caller-owned split-K slab (new; PyTorch autograd allocates internally)",
    "s3od_conv_wgrad_ws": "workspace query of s3od_conv_wgrad: bytes of the caller-owned split-K slab (new; PyTorch autograd allocates internally)",
    "s3od_token_prefix_bwd": "cat([cls, register_tokens, patches]) backward: tf:modeling_dinov3_vit.py:88-92 (reference: implicit torch autograd)",
    "s3od_layernorm_ls_bwd": "norm2 / norm1 LayerNorm backward fused with the DINOv3ViTLayerScale backward that consumes its dx: tf:modeling_dinov3_vit.py:337-343, 419-445 (reference: implicit torch autograd)",
}

# caller-owned buffers whose size is not implied by the other arguments (a non-Python caller sizes them
# from this header).  NREP = S3OD_NREP replicas (#define below).
WS = {
    "s3od_conv_fwd": "stats (nullable): fp64 [S3OD_NREP][2][Cout] (sum | sum of squares replicas), all zero on entry; s3od_bn_finalize folds and clears it",
    "s3od_bn_finalize": "stats: the fp64 [S3OD_NREP][2][C] replicas s3od_conv_fwd filled; read and left all zero",
    "s3od_bn_bwd": "sums: fp64 [S3OD_NREP][3][C], all zero on entry, left all zero",
    "s3od_bn_relu_bwd": "sums: fp64 [S3OD_NREP][3][C], all zero on entry, left all zero",
    "s3od_layernorm_bwd": "ws: fp32 [S3OD_NREP][2][D], all zero on entry, left all zero",
    "s3od_layernorm_ls_bwd": "ws, ws2: fp32 [S3OD_NREP][2][D] each (LayerNorm dw|db and LayerScale dlam|dbias replicas), all zero on entry, left all zero",
    "s3od_layerscale_bwd": "ws: fp32 [S3OD_NREP][2][D], all zero on entry, left all zero",
    "s3od_qkv_unrope": "ws: fp32 [S3OD_NREP][2][64 H], all zero on entry, left all zero",
    "s3od_attn_bwd_qkv": "ws: fp32 [S3OD_NREP][2][64 H], all zero on entry, left all zero",
    "s3od_conv_wgrad": "ws (nullable): fp32 [Cout][KH][KW][Cin], all zero on entry, left all zero; slab (nullable): >= s3od_conv_wgrad_ws bytes, contents dead between calls",
    "s3od_avgpool": "ws: fp32 [B][ceil(HW / 1024)][C] partial sums, contents dead between calls (a fixed-order two-pass mean: deterministic)",
    "s3od_colsum": "ws (nullable): >= s3od_colsum_ws bytes of fp32 partial sums, contents dead between calls (with it the sum is two fixed-order passes: deterministic, no same-address atomics; without it one fp32 atomic per column per block)",
    "s3od_linear_wgrad": "slab (nullable): >= s3od_linear_wgrad_ws bytes, contents dead between calls (without it the split-K partials are fp32 atomics into dw)",
}

SIG = re.compile(r"^(int|const char\*)\s+(s3od_\w+)\(([^)]*)\)\s*\{", re.M | re.S)


def collect():
    out = []
    for f in sorted((ROOT / "s3od_amd" / "csrc").glob("*.hip")):
        txt = f.read_text()
        i = txt.find('extern "C"')
        if i < 0:
            continue
        for m in SIG.finditer(txt, i):
            if m.group(2).startswith("s3od_dbg_"):
                continue                    # dev-build entry points (#ifdef S3OD_TIMELINE), not part of the ABI
            args = " ".join(m.group(3).split())
            out.append((m.group(2), m.group(1), args, f.name))
    return out


def nrep():
    m = re.search(r"constexpr int S3OD_NREP = (\d+);", (ROOT / "s3od_amd" / "csrc" / "common.hpp").read_text())
    return int(m.group(1))


def main():
    decls = collect()
    lines = [
        "/* libs3od_hip.so — C ABI of the MI355X (gfx950) S3OD hot path.",
        " * GENERATED by tools/gen_header.py from s3od_amd/csrc/*.hip; do not edit by hand.",
        " *",
        " * Conventions: device pointers only; the caller (PyTorch caching allocator) owns every",
        " * buffer, workspaces included (sizes stated per entry below or returned by a *_ws query):",
        " * the library never allocates.  `stream` is a hipStream_t.  dtype: 0 = f32 (strict",
        " * parity path, v_mfma_f32_16x16x4_f32), 1 = bf16 (fast path, v_mfma_f32_16x16x32_bf16).",
        " * Activations are NHWC; weights are repacked [Cout][KH][KW][Cin] for the kernels while",
        " * gradients are written in the reference (PyTorch state_dict) layout.",
        " * act (GEMM / conv epilogues): 0 none, 1 ReLU, 2 GELU (erf), 3 x GELU'(res1 = saved pre-activation),",
        " * 4 x ReLU'(res1 = saved output), 5 GELU with gelu'(v) written to `pre`, 6 x res1 (a saved gelu').",
        " * Return: 0 on success, otherwise a hipError_t or 22 (invalid argument);",
        " * s3od_last_error() describes the last failure on the calling thread.",
        " */",
        "#ifndef S3OD_HIP_H",
        "#define S3OD_HIP_H",
        "",
        "/* replicas of the column-sum / BN-statistic accumulation workspaces (sizes below) */",
        f"#define S3OD_NREP {nrep()}",
        "#ifdef __cplusplus",
        'extern "C" {',
        "#endif",
        "",
    ]
    for name, ret, args, src in decls:
        lines.append(f"/* {REF[name]}  [{src}]" + (f"\n * buffers: {WS[name]}" if name in WS else "") + " */")
        lines.append(f"{ret} {name}({args});")
        lines.append("")
    lines += ["#ifdef __cplusplus", "}", "#endif", "#endif  /* S3OD_HIP_H */", ""]
    (ROOT / "include" / "s3od_hip.h").write_text("\n".join(lines))
    print(f"{len(decls)} declarations")


if __name__ == "__main__":
    main()

"""Generate tests/golden/hf_anchor.npz: a structural cross-check of the
encoder/decoder oracle against an independent implementation.

NOT the parity oracle (the reference's numerics are ggml's, restated in
oracle/qasr_oracle.c); this pins what a restatement can get wrong
structurally: the GGUF tensor-name / transpose mapping, the conv feature
order c*16+f (src/audio_encoder.cpp:133-142), the per-chunk sinusoidal PE
restart (:400-404), the projector, NEOX RoPE, q/k RMSNorm, GQA, the audio
splice (src/text_decoder.cpp:431-459) and the tied LM head.

The independent implementation is transformers' `models/qwen3_asr`
(transformers 5.15.0, site-packages; SURVEY.md §8(c) "cross-check only"),
instantiated from a local config -- no download -- and loaded with the
weights of the repo's seeded tiny synthetic GGUF through the inverse of the
reference converter's name map (scripts/convert_hf_to_gguf.py:50-120, with
the transformers port's module names).  Settings that make HF compute the
reference's function:
  * n_window_infer = 10000 mel frames: one attention window per clip = the
    reference's full bidirectional attention (src/audio_encoder.cpp:466-486);
  * mel lengths a multiple of 100 frames: HF's zero-padded chunks equal the
    reference's unpadded ones;
  * activation "gelu_pytorch_tanh": the reference's tanh GELU (ggml_gelu);
    the oracle runs with QO_GELU_EXACT (fp32 tanh GELU instead of the fp16 LUT);
  * the mel is the oracle's (= the reference build's, tests/test_oracle_golden.py),
    fed directly (HF's own feature extractor uses a slaney filterbank).
HF runs in fp32; the oracle rounds matmul inputs to fp16 as ggml does, so
the comparison is a tolerance, not bit-exact (tests/test_hf_anchor.py).

Run in the build container only (transformers + torch CPU):
    python tests/golden/make_hf_anchor.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "qwen3-asr.cpp_amd", "python"))

import oracle_py as op  # noqa: E402
import qasr  # noqa: E402

CLIPS = [(21000, 3.0), (21001, 5.0), (21002, 8.0)]   # (seed, seconds): 300 / 500 / 800 mel frames


def f16(a):
    return np.asarray(a).view(np.float16).astype(np.float32)


def to_torch(g: op.Gguf, name: str) -> torch.Tensor:
    ty, ne, arr = g.tensors[name]
    a = arr.astype(np.float32) if ty == 0 else f16(arr)
    return torch.from_numpy(a.reshape(tuple(reversed(ne))).copy())


def hf_model(g: op.Gguf):
    from transformers import Qwen3ASRConfig, Qwen3ASRForConditionalGeneration
    kv = g.kv
    D = kv["qwen3-asr.audio.encoder.embedding_length"]
    H = kv["qwen3-asr.embedding_length"]
    cfg = Qwen3ASRConfig(
        audio_config=dict(
            num_mel_bins=128, encoder_layers=kv["qwen3-asr.audio.encoder.layer_count"],
            encoder_attention_heads=kv["qwen3-asr.audio.encoder.attention.head_count"],
            encoder_ffn_dim=kv["qwen3-asr.audio.encoder.feed_forward_length"], d_model=D,
            activation_function="gelu_pytorch_tanh", output_dim=H, n_window=50, n_window_infer=10000,
            downsample_hidden_size=kv["qwen3-asr.audio.conv_channels"], max_position_embeddings=13),
        text_config=dict(
            vocab_size=kv["qwen3-asr.vocab_size"], hidden_size=H, intermediate_size=kv["qwen3-asr.feed_forward_length"],
            num_hidden_layers=kv["qwen3-asr.block_count"], num_attention_heads=kv["qwen3-asr.attention.head_count"],
            num_key_value_heads=kv["qwen3-asr.attention.head_count_kv"], head_dim=kv["qwen3-asr.attention.key_length"],
            rms_norm_eps=kv["qwen3-asr.attention.layer_norm_rms_epsilon"], max_position_embeddings=4096,
            rope_parameters={"rope_type": "default", "rope_theta": kv["qwen3-asr.rope.freq_base"]},
            tie_word_embeddings=True, attention_bias=False),
        audio_token_id=kv["qwen3-asr.audio.pad_token_id"], tie_word_embeddings=True)
    cfg._attn_implementation = "eager"
    cfg.audio_config._attn_implementation = "eager"
    cfg.text_config._attn_implementation = "eager"
    m = Qwen3ASRForConditionalGeneration(cfg).float().eval()
    # inverse of scripts/convert_hf_to_gguf.py:50-120 onto the transformers port's modules
    sd = {}
    at, lm = "model.audio_tower.", "model.language_model."
    for i, n in ((1, "conv2d1"), (2, "conv2d2"), (3, "conv2d3")):
        sd[f"{at}{n}.weight"] = f"audio.encoder.conv{i}.weight"
        sd[f"{at}{n}.bias"] = f"audio.encoder.conv{i}.bias"
    sd[f"{at}conv_out.weight"] = "audio.encoder.conv_out.weight"
    for s in ("weight", "bias"):
        sd[f"{at}ln_post.{s}"] = f"audio.encoder.ln_post.{s}"
        sd[f"model.multi_modal_projector.linear_1.{s}"] = f"audio.encoder.proj1.{s}"
        sd[f"model.multi_modal_projector.linear_2.{s}"] = f"audio.encoder.proj2.{s}"
    for l in range(cfg.audio_config.encoder_layers):
        p, q = f"{at}layers.{l}.", f"audio.encoder.blk.{l}."
        for hn, gn in (("self_attn.q_proj", "attn_q"), ("self_attn.k_proj", "attn_k"), ("self_attn.v_proj", "attn_v"),
                       ("self_attn.out_proj", "attn_out"), ("self_attn_layer_norm", "attn_norm"),
                       ("final_layer_norm", "ffn_norm"), ("fc1", "ffn_up"), ("fc2", "ffn_down")):
            for s in ("weight", "bias"):
                sd[f"{p}{hn}.{s}"] = f"{q}{gn}.{s}"
    sd[f"{lm}embed_tokens.weight"] = "token_embd.weight"
    sd[f"{lm}norm.weight"] = "output_norm.weight"
    for l in range(cfg.text_config.num_hidden_layers):
        p, q = f"{lm}layers.{l}.", f"blk.{l}."
        for hn, gn in (("input_layernorm", "attn_norm"), ("self_attn.q_proj", "attn_q"), ("self_attn.k_proj", "attn_k"),
                       ("self_attn.v_proj", "attn_v"), ("self_attn.o_proj", "attn_output"),
                       ("self_attn.q_norm", "attn_q_norm"), ("self_attn.k_norm", "attn_k_norm"),
                       ("post_attention_layernorm", "ffn_norm"), ("mlp.gate_proj", "ffn_gate"),
                       ("mlp.up_proj", "ffn_up"), ("mlp.down_proj", "ffn_down")):
            sd[f"{p}{hn}.weight"] = f"{q}{gn}.weight"
    state = {k: to_torch(g, v) for k, v in sd.items()}
    state["lm_head.weight"] = state[f"{lm}embed_tokens.weight"]
    missing, unexpected = m.load_state_dict(state, strict=False)
    missing = [k for k in missing if not k.endswith("positional_embedding.positional_embedding")]
    assert not missing and not unexpected, (missing, unexpected)
    return m


def main():
    path = os.path.join("/tmp", "hf_anchor_tiny.gguf")
    qasr.write_synthetic_gguf(path, "tiny", 42, 1)
    g = op.Gguf(path)
    m = hf_model(g)
    om = op.OracleModel(path)
    out = {"model": np.array("tiny synthetic GGUF, qasr_write_synthetic_gguf(seed 42, f16)"),
           "transformers_version": np.array(__import__("transformers").__version__)}
    torch.manual_seed(0)
    for i, (seed, secs) in enumerate(CLIPS):
        pcm = qasr.synth_pcm(seed, int(secs * 16000))
        mel = op.log_mel(pcm)
        T = mel.shape[1]
        assert T % 100 == 0, T
        with torch.no_grad():
            feats_in = torch.from_numpy(mel)[None]
            mask = torch.ones(1, T, dtype=torch.long)
            feats = m.model.get_audio_features(feats_in, mask, return_dict=True).pooler_output
            N = feats.shape[0]
            ids = np.asarray(om.prompt(N), np.int32)   # src/qwen3_asr.cpp:151-214 chat template
            logits = m(input_ids=torch.from_numpy(ids.astype(np.int64))[None], input_features=feats_in,
                       input_features_mask=mask).logits[0, -1].numpy()
        top = np.argsort(-logits)[:32]
        out[f"mel{i}"] = mel
        out[f"feats{i}"] = feats.numpy().astype(np.float32)
        out[f"ids{i}"] = ids
        out[f"logits_head{i}"] = logits[:4096].astype(np.float32)
        out[f"logits_top_idx{i}"] = top.astype(np.int32)
        out[f"logits_top_val{i}"] = logits[top].astype(np.float32)
        out[f"logits_absmax{i}"] = np.float32(np.abs(logits).max())
        print(f"clip {i}: T={T} N={N} P={len(ids)} argmax={int(top[0])}", flush=True)
    np.savez_compressed(os.path.join(HERE, "hf_anchor.npz"), **out)


if __name__ == "__main__":
    main()

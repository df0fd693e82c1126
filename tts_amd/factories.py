"""Config loading and model factories with the reference's signatures.

* ``load_config``   <- ``TTS/utils/io.py:12-34`` (JSON with ``//`` comments -> AttrDict)
* ``setup_model``   <- ``TTS/tts/utils/generic_utils.py:48-130`` (Tacotron2 branch)
* ``setup_generator`` <- ``TTS/vocoder/utils/generic_utils.py:45-94`` (MelGAN branches)
"""

import json
import re

from .glow_tts import GlowTts
from .tacotron2 import Tacotron2
from .vocoder import FullbandMelganGenerator, MelganGenerator, MultibandMelganGenerator, ParallelWaveganGenerator


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def load_config(config_path):
    config = AttrDict()
    with open(config_path, "r") as f:
        s = f.read()
    s = re.sub(r"\\\n", "", s)
    s = re.sub(r"//.*\n", "\n", s)
    config.update(json.loads(s))
    return config


def _get(c, k, default=None):
    return c[k] if k in c else default


def setup_model(num_chars, num_speakers, c, speaker_embedding_dim=None):
    print(" > Using model: {}".format(c["model"]))
    if c["model"].lower() == "glow_tts":  # TTS/tts/utils/generic_utils.py:105-129
        return GlowTts(num_chars=num_chars, hidden_channels=192, filter_channels=768, filter_channels_dp=256,
                       out_channels=80, kernel_size=3, num_heads=2, num_layers_enc=6,
                       encoder_type=_get(c, "encoder_type", "gatedconv"), dropout_p=0.1, num_flow_blocks_dec=12,
                       kernel_size_dec=5, dilation_rate=1, num_block_layers=4, dropout_p_dec=0.05,
                       num_speakers=num_speakers, c_in_channels=0, num_splits=4, num_sqz=2, sigmoid_scale=False,
                       mean_only=True, hidden_channels_enc=192, hidden_channels_dec=192, use_encoder_prenet=True)
    if c["model"].lower() != "tacotron2":
        raise NotImplementedError(f"model {c['model']} is outside the MI355X hot path (SURVEY.md §8f)")
    gst = _get(c, "gst", {}) or {}
    return Tacotron2(num_chars=num_chars, num_speakers=num_speakers, r=c["r"],
                     postnet_output_dim=c["audio"]["num_mels"], decoder_output_dim=c["audio"]["num_mels"],
                     gst=_get(c, "use_gst", False), gst_embedding_dim=gst.get("gst_embedding_dim", 512),
                     gst_num_heads=gst.get("gst_num_heads", 4), gst_style_tokens=gst.get("gst_style_tokens", 10),
                     gst_use_speaker_embedding=gst.get("gst_use_speaker_embedding", False),
                     attn_type=_get(c, "attention_type", "original"), attn_win=_get(c, "windowing", False),
                     attn_norm=_get(c, "attention_norm", "softmax"), prenet_type=_get(c, "prenet_type", "original"),
                     prenet_dropout=_get(c, "prenet_dropout", True), forward_attn=_get(c, "use_forward_attn", False),
                     trans_agent=_get(c, "transition_agent", False),
                     forward_attn_mask=_get(c, "forward_attn_mask", False),
                     location_attn=_get(c, "location_attn", True), attn_K=_get(c, "attention_heads", 5),
                     separate_stopnet=_get(c, "separate_stopnet", True),
                     bidirectional_decoder=_get(c, "bidirectional_decoder", False),
                     double_decoder_consistency=_get(c, "double_decoder_consistency", False),
                     ddc_r=_get(c, "ddc_r", None), speaker_embedding_dim=speaker_embedding_dim)


def setup_generator(c):
    name = c["generator_model"]
    print(" > Generator Model: {}".format(name))
    p = c["generator_model_params"]
    n_mels = c["audio"]["num_mels"]
    if name == "melgan_generator":
        return MelganGenerator(in_channels=n_mels, out_channels=1, proj_kernel=7, base_channels=512,
                               upsample_factors=p["upsample_factors"], res_kernel=3,
                               num_res_blocks=p["num_res_blocks"])
    if name == "multiband_melgan_generator":
        return MultibandMelganGenerator(in_channels=n_mels, out_channels=4, proj_kernel=7, base_channels=384,
                                        upsample_factors=p["upsample_factors"], res_kernel=3,
                                        num_res_blocks=p["num_res_blocks"])
    if name == "fullband_melgan_generator":
        return FullbandMelganGenerator(in_channels=n_mels, out_channels=1, proj_kernel=7, base_channels=512,
                                       upsample_factors=p["upsample_factors"], res_kernel=3,
                                       num_res_blocks=p["num_res_blocks"])
    if name == "parallel_wavegan_generator":  # generic_utils.py:79-92
        return ParallelWaveganGenerator(in_channels=1, out_channels=1, kernel_size=3,
                                        num_res_blocks=p["num_res_blocks"], stacks=p["stacks"], res_channels=64,
                                        gate_channels=128, skip_channels=64, aux_channels=n_mels, dropout=0.0,
                                        bias=True, use_weight_norm=True, upsample_factors=p["upsample_factors"])
    raise NotImplementedError(f"generator {name} is outside the MI355X hot path (SURVEY.md §8f)")

"""Parameter specs (state_dict names and shapes) of the two models on the hot path.

The names are the reference checkpoint keys, so a reference ``.pth.tar`` ``['model']``
state_dict loads unchanged:

* Tacotron2: ``TTS/tts/models/tacotron2.py:61-87`` (embedding, encoder, decoder, postnet,
  DDC ``coarse_decoder``), layers from ``TTS/tts/layers/tacotron2.py:9-233`` and
  ``TTS/tts/layers/common_layers.py:6-110,196-263``.
* MultiBand-MelGAN: ``TTS/vocoder/models/melgan_generator.py:28-78`` (``layers.N``),
  ``TTS/vocoder/layers/melgan.py:5-39`` (ResidualStack), ``TTS/vocoder/layers/pqmf.py:34-43``
  (buffers ``H``, ``G``, ``updown_filter``).

Each entry is ``(name, shape, kind)``; ``kind`` is a tag used by the synthetic weight
generator (``tts_amd.weights``) to pick a scale, and by the packers to know what a tensor is.
"""

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

Spec = List[Tuple[str, Tuple[int, ...], str]]


@dataclass
class TacotronConfig:
    """Architecture knobs of ``Tacotron2(...)`` that change tensor shapes or math.

    Defaults follow the DDC LJSpeech config (``TTS/tts/configs/config.json:66-140``):
    r=7 at construction, sigmoid attention norm, location attention, DDC coarse decoder.
    """
    num_chars: int = 129
    r: int = 7                      # r_init: width of linear_projection = 80 * r
    frame_channels: int = 80
    postnet_channels: int = 80
    attn_norm: str = "sigmoid"      # 'sigmoid' | 'softmax'  (common_layers.py:347-354)
    location_attn: bool = True
    double_decoder_consistency: bool = True
    ddc_r: int = 7
    encoder_dim: int = 512
    query_dim: int = 1024
    decoder_rnn_dim: int = 1024
    prenet_dim: int = 256
    attn_dim: int = 128
    loc_filters: int = 32
    loc_kernel: int = 31
    # multi-speaker (models/tacotron2.py:50-58): num_speakers > 1 concatenates a speaker vector to
    # every encoder output; a learned nn.Embedding(num_speakers, 512) unless speaker_embedding_dim
    # is given (external per-sample embeddings, tacotron_abstract.py:76-81)
    num_speakers: int = 0
    speaker_embedding_dim: Optional[int] = None
    # decoder variants (layers/tacotron2.py:147-200, common_layers.py:49-74,196-372)
    prenet_type: str = "original"   # 'original' | 'bn' (LinearBN: Linear(bias=False) + BatchNorm1d)
    windowing: bool = False         # attention windowing at inference (common_layers.py:286-300)
    forward_attn: bool = False      # forward attention (common_layers.py:302-323)
    trans_agent: bool = False       # transition agent u = sigmoid(ta([ctx, query]))
    forward_attn_mask: bool = False  # forward attention kept to [n-1, n+2] (common_layers.py:309-318)
    attn_type: str = "original"     # or "graves" (GravesAttention, common_layers.py:113-193)
    bidirectional_decoder: bool = False  # decoder_backward: a training-time copy, unused at inference
    attn_K: int = 5                 # Graves mixture components

    @property
    def spk_dim(self) -> int:
        if self.num_speakers <= 1:
            return 0
        return 512 if self.speaker_embedding_dim is None else int(self.speaker_embedding_dim)

    @property
    def decoder_in(self) -> int:
        """decoder_in_features (models/tacotron2.py:57-58)."""
        return self.encoder_dim + self.spk_dim


@dataclass
class MelganConfig:
    """``MultibandMelganGenerator`` constructor args as ``setup_generator`` passes them
    (``TTS/vocoder/utils/generic_utils.py:61-69``; MB config ``multiband_melgan_config.json:83-87``)."""
    in_channels: int = 80
    out_channels: int = 4
    proj_kernel: int = 7
    base_channels: int = 384
    upsample_factors: Tuple[int, ...] = (8, 4, 2)
    res_kernel: int = 3
    num_res_blocks: int = 4
    pqmf: bool = True
    pqmf_taps: int = 62
    pqmf_cutoff: float = 0.15
    pqmf_beta: float = 9.0


def _conv_bn(prefix: str, cin: int, cout: int, k: int) -> Spec:
    return [
        (f"{prefix}.convolution1d.weight", (cout, cin, k), "conv"),
        (f"{prefix}.convolution1d.bias", (cout,), "bias"),
        (f"{prefix}.batch_normalization.weight", (cout,), "bn_w"),
        (f"{prefix}.batch_normalization.bias", (cout,), "bn_b"),
        (f"{prefix}.batch_normalization.running_mean", (cout,), "bn_mean"),
        (f"{prefix}.batch_normalization.running_var", (cout,), "bn_var"),
        (f"{prefix}.batch_normalization.num_batches_tracked", (), "count"),
    ]


def _decoder(prefix: str, c: TacotronConfig, r: int) -> Spec:
    E, Q, D, P, A = c.decoder_in, c.query_dim, c.decoder_rnn_dim, c.prenet_dim, c.attn_dim
    F = c.frame_channels
    s: Spec = []
    for i, din in enumerate((F, P)):
        s.append((f"{prefix}.prenet.linear_layers.{i}.linear_layer.weight", (P, din), "linear_relu"))
        if c.prenet_type == "bn":
            bn = f"{prefix}.prenet.linear_layers.{i}.batch_normalization"
            s += [(f"{bn}.weight", (P,), "bn_w"), (f"{bn}.bias", (P,), "bn_b"),
                  (f"{bn}.running_mean", (P,), "bn_mean"), (f"{bn}.running_var", (P,), "bn_var"),
                  (f"{bn}.num_batches_tracked", (), "count")]
    s += [
        (f"{prefix}.attention_rnn.weight_ih", (4 * Q, P + E), "lstm"),
        (f"{prefix}.attention_rnn.weight_hh", (4 * Q, Q), "lstm"),
        (f"{prefix}.attention_rnn.bias_ih", (4 * Q,), "lstm"),
        (f"{prefix}.attention_rnn.bias_hh", (4 * Q,), "lstm"),
    ]
    if c.attn_type == "graves":  # N_a = Linear(Q, Q) -> ReLU -> Linear(Q, 3K)
        s += [(f"{prefix}.attention.N_a.0.weight", (Q, Q), "linear_relu"),
              (f"{prefix}.attention.N_a.0.bias", (Q,), "bias"),
              (f"{prefix}.attention.N_a.2.weight", (3 * c.attn_K, Q), "linear"),
              (f"{prefix}.attention.N_a.2.bias", (3 * c.attn_K,), "bias")]
    else:  # OriginalAttention (common_layers.py:196-232)
        s += [
            (f"{prefix}.attention.query_layer.linear_layer.weight", (A, Q), "linear_tanh"),
            (f"{prefix}.attention.inputs_layer.linear_layer.weight", (A, E), "linear_tanh"),
            (f"{prefix}.attention.v.linear_layer.weight", (1, A), "attn_v"),
            (f"{prefix}.attention.v.linear_layer.bias", (1,), "bias"),
        ]
        if c.forward_attn and c.trans_agent:
            s += [(f"{prefix}.attention.ta.weight", (1, Q + E), "linear_sigmoid"),
                  (f"{prefix}.attention.ta.bias", (1,), "bias")]
        if c.location_attn:
            s += [
                (f"{prefix}.attention.location_layer.location_conv1d.weight",
                 (c.loc_filters, 2, c.loc_kernel), "conv"),
                (f"{prefix}.attention.location_layer.location_dense.linear_layer.weight",
                 (A, c.loc_filters), "linear_tanh"),
            ]
    s += [
        (f"{prefix}.decoder_rnn.weight_ih", (4 * D, Q + E), "lstm"),
        (f"{prefix}.decoder_rnn.weight_hh", (4 * D, D), "lstm"),
        (f"{prefix}.decoder_rnn.bias_ih", (4 * D,), "lstm"),
        (f"{prefix}.decoder_rnn.bias_hh", (4 * D,), "lstm"),
        (f"{prefix}.linear_projection.linear_layer.weight", (F * r, D + E), "linear"),
        (f"{prefix}.linear_projection.linear_layer.bias", (F * r,), "bias"),
        (f"{prefix}.stopnet.1.linear_layer.weight", (1, D + F * r), "linear_sigmoid"),
        (f"{prefix}.stopnet.1.linear_layer.bias", (1,), "stop_bias"),
    ]
    return s


def tacotron2_spec(c: TacotronConfig) -> Spec:
    """Ordered state_dict spec of ``Tacotron2`` (no GST)."""
    E = c.encoder_dim
    s: Spec = []
    if c.num_speakers > 1 and c.speaker_embedding_dim is None:
        s.append(("speaker_embedding.weight", (c.num_speakers, 512), "speaker_emb"))
    s.append(("embedding.weight", (c.num_chars, E), "embedding"))
    for i in range(3):
        s += _conv_bn(f"encoder.convolutions.{i}", E, E, 5)
    H = E // 2
    for sfx in ("", "_reverse"):
        s += [
            (f"encoder.lstm.weight_ih_l0{sfx}", (4 * H, E), "lstm_enc"),
            (f"encoder.lstm.weight_hh_l0{sfx}", (4 * H, H), "lstm_enc"),
            (f"encoder.lstm.bias_ih_l0{sfx}", (4 * H,), "lstm_enc"),
            (f"encoder.lstm.bias_hh_l0{sfx}", (4 * H,), "lstm_enc"),
        ]
    s += _decoder("decoder", c, c.r)
    F = c.postnet_channels
    chans = [F, 512, 512, 512, 512, F]
    for i in range(5):
        s += _conv_bn(f"postnet.convolutions.{i}", chans[i], chans[i + 1], 5)
    if c.bidirectional_decoder:  # tacotron_abstract.py:104-105 (deepcopy of the decoder)
        s += _decoder("decoder_backward", c, c.r)
    if c.double_decoder_consistency:
        s += _decoder("coarse_decoder", c, c.ddc_r)
    return s


@dataclass
class MelganLayer:
    """One weight-bearing op of the generator, in execution order."""
    kind: str            # 'conv_in' | 'convT' | 'res_dconv' | 'res_1x1' | 'res_sc' | 'conv_out'
    name: str            # state_dict prefix, e.g. 'layers.4.blocks.0.2'
    cin: int
    cout: int
    k: int
    stride: int = 1
    dilation: int = 1
    padding: int = 0
    transposed: bool = False
    extra: dict = field(default_factory=dict)


def melgan_layers(c: MelganConfig) -> List[MelganLayer]:
    """Generator topology (melgan_generator.py:28-78, melgan.py:9-33)."""
    L: List[MelganLayer] = []
    pad = (c.proj_kernel - 1) // 2
    L.append(MelganLayer("conv_in", "layers.1", c.in_channels, c.base_channels, c.proj_kernel,
                         padding=pad))
    idx = 2
    cout = c.base_channels
    for i, u in enumerate(c.upsample_factors):
        cin = c.base_channels // (2 ** i)
        cout = c.base_channels // (2 ** (i + 1))
        op = u % 2
        p = u // 2 + op
        # layers[idx] = LeakyReLU, layers[idx+1] = ConvTranspose1d, layers[idx+2] = ResidualStack
        L.append(MelganLayer("convT", f"layers.{idx + 1}", cin, cout, 2 * u, stride=u, padding=p,
                             transposed=True, extra={"output_padding": op}))
        base_pad = (c.res_kernel - 1) // 2
        for b in range(c.num_res_blocks):
            d = c.res_kernel ** b
            L.append(MelganLayer("res_dconv", f"layers.{idx + 2}.blocks.{b}.2", cout, cout,
                                 c.res_kernel, dilation=d, padding=base_pad * d))
            L.append(MelganLayer("res_1x1", f"layers.{idx + 2}.blocks.{b}.4", cout, cout, 1))
            L.append(MelganLayer("res_sc", f"layers.{idx + 2}.shortcuts.{b}", cout, cout, 1))
        idx += 3
    # layers[idx] = LeakyReLU, [idx+1] = ReflectionPad, [idx+2] = Conv, [idx+3] = Tanh
    L.append(MelganLayer("conv_out", f"layers.{idx + 2}", cout, c.out_channels, c.proj_kernel,
                         padding=pad))
    return L


def melgan_spec(c: MelganConfig, weight_norm: bool = True) -> Spec:
    """Ordered state_dict spec; ``weight_norm=True`` is the checkpoint (pre-removal) naming."""
    s: Spec = []
    for l in melgan_layers(c):
        wshape = (l.cin, l.cout, l.k) if l.transposed else (l.cout, l.cin, l.k)
        s.append((f"{l.name}.bias", (l.cout,), "bias"))
        if weight_norm:
            s.append((f"{l.name}.weight_g", (wshape[0], 1, 1), "wn_g"))
            s.append((f"{l.name}.weight_v", wshape, "conv"))
        else:
            s.append((f"{l.name}.weight", wshape, "conv"))
    if c.pqmf:
        N, taps = c.out_channels, c.pqmf_taps
        s += [("pqmf_layer.H", (N, 1, taps + 1), "buffer"),
              ("pqmf_layer.G", (1, N, taps + 1), "buffer"),
              ("pqmf_layer.updown_filter", (N, N, N), "buffer")]
    return s


@dataclass
class Ge2eConfig:
    """``SpeakerEncoder(input_dim, proj_dim, lstm_dim, num_lstm_layers, use_lstm_with_projection)``
    (``TTS/speaker_encoder/model.py:31-47``; config ``speaker_encoder/config.json:47-52``)."""
    input_dim: int = 40
    proj_dim: int = 256
    lstm_dim: int = 768
    num_lstm_layers: int = 3
    use_lstm_with_projection: bool = True


def ge2e_spec(c: Ge2eConfig) -> Spec:
    """state_dict spec of ``SpeakerEncoder``: ``layers.{i}.lstm.*_l0`` + ``layers.{i}.linear.weight``
    (LSTMWithProjection, model.py:5-17) or ``layers.lstm.*_l{k}`` + ``layers.linear.{weight,bias}``
    (LSTMWithoutProjection, model.py:19-30)."""
    H, P = c.lstm_dim, c.proj_dim
    s: Spec = []
    if c.use_lstm_with_projection:
        for i in range(c.num_lstm_layers):
            din = c.input_dim if i == 0 else P
            s += [
                (f"layers.{i}.lstm.weight_ih_l0", (4 * H, din), "xavier"),
                (f"layers.{i}.lstm.weight_hh_l0", (4 * H, H), "xavier"),
                (f"layers.{i}.lstm.bias_ih_l0", (4 * H,), "bias"),
                (f"layers.{i}.lstm.bias_hh_l0", (4 * H,), "bias"),
                (f"layers.{i}.linear.weight", (P, H), "xavier"),
            ]
    else:
        for k in range(c.num_lstm_layers):
            din = c.input_dim if k == 0 else H
            s += [
                (f"layers.lstm.weight_ih_l{k}", (4 * H, din), "xavier"),
                (f"layers.lstm.weight_hh_l{k}", (4 * H, H), "xavier"),
                (f"layers.lstm.bias_ih_l{k}", (4 * H,), "bias"),
                (f"layers.lstm.bias_hh_l{k}", (4 * H,), "bias"),
            ]
        s += [("layers.linear.weight", (P, H), "xavier"), ("layers.linear.bias", (P,), "bias")]
    return s


@dataclass
class GlowConfig:
    """``GlowTts`` as ``setup_model`` builds it for the reference configs
    (``TTS/tts/utils/generic_utils.py:105-129``; ``configs/glow_tts_gated_conv.json``): hidden 192,
    duration-predictor filters 256, 80 mel channels, gated-conv encoder with 3 + 6 layers, 12 flow
    blocks of 4 WN layers (kernel 5, dilation 1), num_sqz 2, num_splits 4, mean_only."""
    num_chars: int = 129
    hidden_channels: int = 192
    filter_channels_dp: int = 256
    out_channels: int = 80
    num_layers_enc: int = 6
    filter_channels: int = 768       # transformer FFN width
    encoder_type: str = "gatedconv"  # "time-depth-separable" (configs/glow_tts_tdsep.json), "transformer"
    num_flow_blocks_dec: int = 12
    num_block_layers: int = 4
    kernel_size_dec: int = 5
    # speaker conditioning (glow_tts.py:97-99, encoder.py:112-114,131-135, glow.py:87-91,119-130):
    # emb_g (num_speakers, c_in) when num_speakers > 1; c_in extra duration-predictor input channels
    # and a weight-normed cond_layer (c_in -> 2 H L) per coupling block when c_in > 0
    num_speakers: int = 0
    c_in_channels: int = 0


def glow_spec(c: GlowConfig) -> Spec:
    """state_dict spec of ``GlowTts`` (encoder_type 'gatedconv'): ``encoder.*`` from
    ``layers/glow_tts/encoder.py:59-104`` + ``gated_conv.py`` + ``duration_predictor.py``,
    ``decoder.flows.*`` from ``layers/glow_tts/decoder.py:60-79`` + ``glow.py`` + ``normalization.py``."""
    H, F, C = c.hidden_channels, c.filter_channels_dp, c.out_channels
    s: Spec = [("encoder.emb.weight", (c.num_chars, H), "glow_emb")]
    if c.encoder_type in ("time-depth-separable", "transformer"):
        # ConvLayerNorm prenet (glow.py:8-50; setup_model passes use_encoder_prenet=True)
        for i in range(3):
            s += [(f"encoder.pre.conv_layers.{i}.weight", (H, H, 5), "conv"),
                  (f"encoder.pre.conv_layers.{i}.bias", (H,), "bias")]
        for i in range(3):
            s += [(f"encoder.pre.norm_layers.{i}.gamma", (1, H, 1), "ln_g"),
                  (f"encoder.pre.norm_layers.{i}.beta", (1, H, 1), "bias")]
        s += [("encoder.pre.proj.weight", (H, H, 1), "conv"), ("encoder.pre.proj.bias", (H,), "bias")]

        def bn(name, n):
            return [(f"{name}.weight", (n,), "bn_w"), (f"{name}.bias", (n,), "bn_b"),
                    (f"{name}.running_mean", (n,), "bn_mean"), (f"{name}.running_var", (n,), "bn_var"),
                    (f"{name}.num_batches_tracked", (), "count")]
    if c.encoder_type == "transformer":
        # Transformer (glow_tts/transformer.py:265-319), no relative-position tables (setup_model
        # passes no rel_attn_window_size), FFN kernel 3, filter 768
        L, Fc = c.num_layers_enc, c.filter_channels
        for i in range(L):
            for n in ("q", "k", "v", "o"):
                s += [(f"encoder.encoder.attn_layers.{i}.conv_{n}.weight", (H, H, 1), "xavier"),
                      (f"encoder.encoder.attn_layers.{i}.conv_{n}.bias", (H,), "bias")]
        for i in range(L):
            s += [(f"encoder.encoder.norm_layers_1.{i}.gamma", (1, H, 1), "ln_g"),
                  (f"encoder.encoder.norm_layers_1.{i}.beta", (1, H, 1), "bias")]
        for i in range(L):
            s += [(f"encoder.encoder.ffn_layers.{i}.conv_1.weight", (Fc, H, 3), "conv"),
                  (f"encoder.encoder.ffn_layers.{i}.conv_1.bias", (Fc,), "bias"),
                  (f"encoder.encoder.ffn_layers.{i}.conv_2.weight", (H, Fc, 3), "conv"),
                  (f"encoder.encoder.ffn_layers.{i}.conv_2.bias", (H,), "bias")]
        for i in range(L):
            s += [(f"encoder.encoder.norm_layers_2.{i}.gamma", (1, H, 1), "ln_g"),
                  (f"encoder.encoder.norm_layers_2.{i}.beta", (1, H, 1), "bias")]
    elif c.encoder_type == "time-depth-separable":
        for i in range(3 + c.num_layers_enc):
            q = f"encoder.encoder.layers.{i}"
            s += [(f"{q}.time_conv.weight", (2 * H, H, 1), "conv"), (f"{q}.time_conv.bias", (2 * H,), "bias")]
            s += bn(f"{q}.norm1", 2 * H)
            s += [(f"{q}.depth_conv.weight", (H, 1, 5), "dwconv"), (f"{q}.depth_conv.bias", (H,), "bias")]
            s += bn(f"{q}.norm2", H)
            s += [(f"{q}.time_conv2.weight", (H, H, 1), "conv"), (f"{q}.time_conv2.bias", (H,), "bias")]
            s += bn(f"{q}.norm3", H)
    else:
        for i in range(3 + c.num_layers_enc):
            s += [(f"encoder.encoder.conv_layers.{i}.weight", (2 * H, H, 5), "conv"),
                  (f"encoder.encoder.conv_layers.{i}.bias", (2 * H,), "bias"),
                  (f"encoder.encoder.norm_layers.{i}.gamma", (1, 2 * H, 1), "ln_g"),
                  (f"encoder.encoder.norm_layers.{i}.beta", (1, 2 * H, 1), "bias")]
    dp = "encoder.duration_predictor"
    s += [("encoder.proj_m.weight", (C, H, 1), "conv"), ("encoder.proj_m.bias", (C,), "bias"),
          (f"{dp}.conv_1.weight", (F, H + c.c_in_channels, 3), "conv"), (f"{dp}.conv_1.bias", (F,), "bias"),
          (f"{dp}.norm_1.gamma", (1, F, 1), "ln_g"), (f"{dp}.norm_1.beta", (1, F, 1), "bias"),
          (f"{dp}.conv_2.weight", (F, F, 3), "conv"), (f"{dp}.conv_2.bias", (F,), "bias"),
          (f"{dp}.norm_2.gamma", (1, F, 1), "ln_g"), (f"{dp}.norm_2.beta", (1, F, 1), "bias"),
          (f"{dp}.proj.weight", (1, F, 1), "conv"), (f"{dp}.proj.bias", (1,), "bias")]
    C2 = 2 * C
    for k in range(c.num_flow_blocks_dec):
        f = f"decoder.flows.{3 * k}"
        s += [(f"{f}.logs", (1, C2, 1), "actnorm"), (f"{f}.bias", (1, C2, 1), "bias")]
        s += [(f"decoder.flows.{3 * k + 1}.weight", (4, 4), "orthogonal")]
        f = f"decoder.flows.{3 * k + 2}"
        s += [(f"{f}.start.bias", (H,), "bias"), (f"{f}.start.weight_g", (H, 1, 1), "wn_g"),
              (f"{f}.start.weight_v", (H, C, 1), "conv"),
              (f"{f}.end.weight", (C2, H, 1), "glow_end"), (f"{f}.end.bias", (C2,), "bias")]
        for i in range(c.num_block_layers):
            s += [(f"{f}.wn.in_layers.{i}.bias", (2 * H,), "bias"),
                  (f"{f}.wn.in_layers.{i}.weight_g", (2 * H, 1, 1), "wn_g"),
                  (f"{f}.wn.in_layers.{i}.weight_v", (2 * H, H, c.kernel_size_dec), "conv")]
        for i in range(c.num_block_layers):
            rs = H if i == c.num_block_layers - 1 else 2 * H
            s += [(f"{f}.wn.res_skip_layers.{i}.bias", (rs,), "bias"),
                  (f"{f}.wn.res_skip_layers.{i}.weight_g", (rs, 1, 1), "wn_g"),
                  (f"{f}.wn.res_skip_layers.{i}.weight_v", (rs, H, 1), "conv")]
        if c.c_in_channels:
            L2 = 2 * H * c.num_block_layers
            s += [(f"{f}.wn.cond_layer.bias", (L2,), "bias"), (f"{f}.wn.cond_layer.weight_g", (L2, 1, 1), "wn_g"),
                  (f"{f}.wn.cond_layer.weight_v", (L2, c.c_in_channels, 1), "conv")]
    if c.num_speakers > 1:
        s.append(("emb_g.weight", (c.num_speakers, c.c_in_channels), "glow_spk"))
    return s


@dataclass
class PwganConfig:
    """``ParallelWaveganGenerator`` as ``setup_generator`` builds it
    (``TTS/vocoder/utils/generic_utils.py:79-92``, ``configs/parallel_wavegan_config.json:84-88``):
    30 WaveNet residual blocks in 3 stacks (dilation 2 ** (i % 10)), kernel 3, res / skip 64,
    gate 128, aux 80, weight norm, ConvUpsample 4 x 4 x 4 x 4, inference_padding 2."""
    num_res_blocks: int = 30
    stacks: int = 3
    kernel_size: int = 3
    res_channels: int = 64
    gate_channels: int = 128
    skip_channels: int = 64
    aux_channels: int = 80
    upsample_factors: Tuple[int, ...] = (4, 4, 4, 4)
    inference_padding: int = 2

    def dilation(self, i: int) -> int:
        return 2 ** (i % (self.num_res_blocks // self.stacks))


def pwgan_spec(c: PwganConfig, weight_norm: bool = True) -> Spec:
    """state_dict spec (``parallel_wavegan_generator.py:47-88``, ``layers/parallel_wavegan.py:29-54``,
    ``layers/upsample.py:33-92``); ``weight_norm=True`` is the checkpoint naming (bias, weight_g,
    weight_v per conv, torch.nn.utils.weight_norm dim 0)."""
    s: Spec = []

    def conv(name, shape, bias):
        if bias:
            s.append((f"{name}.bias", (shape[0],), "bias"))
        if weight_norm:
            s.append((f"{name}.weight_g", (shape[0],) + (1,) * (len(shape) - 1), "wn_g"))
            s.append((f"{name}.weight_v", shape, "conv"))
        else:
            s.append((f"{name}.weight", shape, "conv"))

    R, G, S, A = c.res_channels, c.gate_channels, c.skip_channels, c.aux_channels
    conv("first_conv", (R, 1, 1), True)
    conv("upsample_net.conv_in", (A, A, 1), False)
    for i, u in enumerate(c.upsample_factors):
        conv(f"upsample_net.upsample.up_layers.{2 * i + 1}", (1, 1, 1, 2 * u + 1), False)
    for i in range(c.num_res_blocks):
        p = f"conv_layers.{i}."
        conv(p + "conv", (G, R, c.kernel_size), True)
        conv(p + "conv1x1_aux", (G, A, 1), False)
        conv(p + "conv1x1_out", (R, G // 2, 1), True)
        conv(p + "conv1x1_skip", (S, G // 2, 1), True)
    conv("last_conv_layers.1", (S, S, 1), True)
    conv("last_conv_layers.3", (1, S, 1), True)
    return s

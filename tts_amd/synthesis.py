"""The notebook / CLI inference surface of ``TTS/tts/utils/synthesis.py`` over the drop-in models.

``synthesis(model, text, CONFIG, use_cuda, ap, ...)`` returns what the reference returns
(``wav, alignment, decoder_output, postnet_output, stop_tokens, inputs``, ``synthesis.py:178-262``)
for ``tts_amd`` Tacotron2 and GlowTts models; the model call is ``run_model_torch``
(``:48-67``). Host glue only: the model runs in ``libttship.so``; Griffin-Lim (``use_griffin_lim``)
is the CPU fallback of ``tts_amd.audio``. The TF / TFLite backends are outside this build.
"""

import numpy as np
import torch

from .text import text_to_seqvec as _text_to_seqvec


def text_to_seqvec(text, CONFIG, phonemize=None):
    """synthesis.py:10-21 (phonemes need a caller-supplied ``phonemize``: phonemizer is absent)."""
    return np.asarray(_text_to_seqvec(text, CONFIG, phonemize), dtype=np.int32)


def numpy_to_torch(np_array, dtype, cuda=False):
    if np_array is None:
        return None
    tensor = torch.as_tensor(np_array, dtype=dtype)
    return tensor.cuda() if cuda else tensor


def id_to_torch(speaker_id, cuda=False):
    if speaker_id is not None:
        speaker_id = torch.from_numpy(np.asarray(speaker_id)).unsqueeze(0)
    if cuda:
        return speaker_id.cuda()
    return speaker_id


def embedding_to_torch(speaker_embedding, cuda=False):
    if speaker_embedding is not None:
        speaker_embedding = torch.from_numpy(np.asarray(speaker_embedding)).unsqueeze(0).type(torch.FloatTensor)
    if cuda:
        return speaker_embedding.cuda()
    return speaker_embedding


def _get(c, k, default=None):
    try:
        return c[k]
    except (KeyError, TypeError):
        return getattr(c, k, default)


def run_model_torch(model, inputs, CONFIG, truncated, speaker_id=None, style_mel=None, speaker_embeddings=None):
    """synthesis.py:48-67."""
    name = str(_get(CONFIG, "model", "")).lower()
    if "tacotron" in name:
        if truncated:
            # the reference's Tacotron2.inference_truncated calls Encoder.inference_truncated, which
            # does not exist (layers/tacotron2.py:74-119): it raises there, and so does this build
            raise AttributeError("'Encoder' object has no attribute 'inference_truncated'")
        if _get(CONFIG, "use_gst", False):
            return model.inference(inputs, style_mel=style_mel, speaker_ids=speaker_id,
                                   speaker_embeddings=speaker_embeddings)
        return model.inference(inputs, speaker_ids=speaker_id, speaker_embeddings=speaker_embeddings)
    if "glow" in name:
        inputs_lengths = torch.tensor(inputs.shape[1:2]).to(inputs.device)
        postnet_output, _, _, _, alignments, _, _ = model.inference(inputs, inputs_lengths)
        return None, postnet_output.permute(0, 2, 1), alignments, None
    raise NotImplementedError(f"model {name} is outside the MI355X hot path")


def parse_outputs_torch(postnet_output, decoder_output, alignments, stop_tokens):
    """synthesis.py:108-113."""
    postnet_output = postnet_output[0].data.cpu().numpy()
    decoder_output = None if decoder_output is None else decoder_output[0].data.cpu().numpy()
    alignment = alignments[0].cpu().data.numpy()
    stop_tokens = None if stop_tokens is None else stop_tokens[0].cpu().numpy()
    return postnet_output, decoder_output, alignment, stop_tokens


def trim_silence(wav, ap):
    return wav[:ap.find_endpoint(wav)]


def inv_spectrogram(postnet_output, ap, CONFIG):
    if str(_get(CONFIG, "model", "")).lower() in ["tacotron"]:
        return ap.inv_spectrogram(postnet_output.T)
    return ap.inv_melspectrogram(postnet_output.T)


def apply_griffin_lim(inputs, input_lens, CONFIG, ap):
    """synthesis.py:163-177: per sample, cut to (len - 1) hops."""
    wavs = []
    for idx, spec in enumerate(inputs):
        wav_len = (input_lens[idx] * ap.hop_length) - ap.hop_length
        wavs.append(inv_spectrogram(spec, ap, CONFIG)[:wav_len])
    return wavs


def synthesis(model, text, CONFIG, use_cuda, ap, speaker_id=None, style_wav=None, truncated=False,
              enable_eos_bos_chars=False, use_griffin_lim=False, do_trim_silence=False, speaker_embedding=None,
              backend="torch", phonemize=None):  # pylint: disable=unused-argument
    """synthesis.py:178-262 (torch backend)."""
    if backend != "torch":
        raise NotImplementedError("the TF / TFLite backends are outside the MI355X build")
    if _get(CONFIG, "use_gst", False) and style_wav is not None:
        raise NotImplementedError("GST style conditioning is outside the MI355X hot path (SURVEY.md §2)")
    inputs = text_to_seqvec(text, CONFIG, phonemize)
    if speaker_id is not None:
        speaker_id = id_to_torch(speaker_id, cuda=use_cuda)
    if speaker_embedding is not None:
        speaker_embedding = embedding_to_torch(speaker_embedding, cuda=use_cuda)
    inputs = numpy_to_torch(inputs, torch.long, cuda=use_cuda).unsqueeze(0)
    decoder_output, postnet_output, alignments, stop_tokens = run_model_torch(
        model, inputs, CONFIG, truncated, speaker_id, None, speaker_embeddings=speaker_embedding)
    postnet_output, decoder_output, alignment, stop_tokens = parse_outputs_torch(
        postnet_output, decoder_output, alignments, stop_tokens)
    wav = None
    if use_griffin_lim:
        wav = inv_spectrogram(postnet_output, ap, CONFIG)
        if do_trim_silence:
            wav = trim_silence(wav, ap)
    return wav, alignment, decoder_output, postnet_output, stop_tokens, inputs

"""``python -m tts_amd.synthesize TEXT CONFIG MODEL OUT_DIR [--vocoder_path ...]``: the CLI of
``TTS/bin/synthesize.py`` over the drop-in models (same arguments, same output file naming, RTF
printout). The model runs in ``libttship.so``; without a vocoder, Griffin-Lim on the CPU.

Deliberate differences: ``--speaker_fileid`` may be omitted for a single-speaker model (the
reference calls ``None.isdigit()`` there, ``synthesize.py:147-151``); GST style input is outside
this build.
"""

import argparse
import json
import os
import string
import time

import torch

from .audio import AudioProcessor
from .factories import load_config, setup_generator, setup_model
from .synthesis import synthesis
from .text import make_symbols, phonemes, symbols


def tts(model, vocoder_model, text, CONFIG, use_cuda, ap, use_gl, speaker_fileid, speaker_embedding=None):
    """synthesize.py:21-43."""
    t_1 = time.time()
    waveform, _, _, mel_postnet_spec, _, _ = synthesis(model, text, CONFIG, use_cuda, ap, speaker_fileid, None,
                                                       False, CONFIG.get("enable_eos_bos_chars", False), use_gl,
                                                       speaker_embedding=speaker_embedding)
    if not use_gl:
        waveform = vocoder_model.inference(torch.FloatTensor(mel_postnet_spec.T).unsqueeze(0).to(
            next(vocoder_model.parameters()).device)).cpu().numpy()
    waveform = waveform.squeeze()
    rtf = (time.time() - t_1) / (len(waveform) / ap.sample_rate)
    print(" > Run-time: {}".format(time.time() - t_1))
    print(" > Real-time factor: {}".format(rtf))
    print(" > Time per step: {}".format((time.time() - t_1) / len(waveform)))
    return waveform


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("text", type=str)
    parser.add_argument("config_path", type=str)
    parser.add_argument("model_path", type=str)
    parser.add_argument("out_path", type=str)
    parser.add_argument("--use_cuda", type=bool, default=True)
    parser.add_argument("--vocoder_path", type=str, default="")
    parser.add_argument("--vocoder_config_path", type=str, default="")
    parser.add_argument("--batched_vocoder", type=bool, default=True)
    parser.add_argument("--speakers_json", type=str, default="")
    parser.add_argument("--speaker_fileid", type=str, default=None)
    parser.add_argument("--gst_style", default=None)
    args = parser.parse_args(argv)

    C = load_config(args.config_path)
    C["forward_attn_mask"] = True  # synthesize.py:96
    ap = AudioProcessor(**C["audio"])
    syms, phs = symbols, phonemes
    if "characters" in C:
        syms, phs = make_symbols(**C["characters"])
    speaker_embedding, speaker_embedding_dim, num_speakers = None, None, 0
    external = C.get("use_external_speaker_embedding_file", False)
    if args.speakers_json != "":
        speaker_mapping = json.load(open(args.speakers_json, "r"))
        num_speakers = len(speaker_mapping)
        if external:
            key = args.speaker_fileid if args.speaker_fileid is not None else list(speaker_mapping.keys())[0]
            speaker_embedding = speaker_mapping[key]["embedding"]
            speaker_embedding_dim = len(speaker_embedding)
    num_chars = len(phs) if C.get("use_phonemes", False) else len(syms)
    model = setup_model(num_chars, num_speakers, C, speaker_embedding_dim)
    cp = torch.load(args.model_path, map_location=torch.device("cpu"), weights_only=True)
    model.load_state_dict(cp["model"])
    model.eval()
    if args.use_cuda:
        model.cuda()
    if "r" in cp and hasattr(model, "decoder") and hasattr(model.decoder, "set_r"):
        model.decoder.set_r(cp["r"])
    vocoder_model = None
    if args.vocoder_path != "":
        VC = load_config(args.vocoder_config_path)
        vocoder_model = setup_generator(VC)
        vocoder_model.load_state_dict(torch.load(args.vocoder_path, map_location="cpu", weights_only=True)["model"])
        vocoder_model.remove_weight_norm()
        if args.use_cuda:
            vocoder_model.cuda()
        vocoder_model.eval()
    use_griffin_lim = args.vocoder_path == ""
    print(" > Text: {}".format(args.text))
    sid = None
    if not external and args.speaker_fileid is not None and args.speaker_fileid.isdigit():
        sid = int(args.speaker_fileid)
    if args.gst_style is not None:
        raise NotImplementedError("GST style input is outside the MI355X hot path (SURVEY.md §2)")
    wav = tts(model, vocoder_model, args.text, C, args.use_cuda, ap, use_griffin_lim, sid,
              speaker_embedding=speaker_embedding)
    file_name = args.text.replace(" ", "_")
    file_name = file_name.translate(str.maketrans("", "", string.punctuation.replace("_", ""))) + ".wav"
    out_path = os.path.join(args.out_path, file_name)
    print(" > Saving output to {}".format(out_path))
    ap.save_wav(wav, out_path)
    return out_path


if __name__ == "__main__":
    main()

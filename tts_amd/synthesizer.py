"""Batched `Synthesizer.tts` with the reference's constructor, loaders and output.

Follows `TTS/server/synthesizer.py:21-193`. What differs on purpose:
  * all sentences of one `tts()` call decode in ONE batched Tacotron2 call and ONE batched
    vocoder call (the reference loops B=1 per sentence, because its decoder cannot batch,
    `TTS/tts/layers/tacotron2.py:362`); per-sentence outputs are cut back to each sentence's
    own mel length, so every sentence equals its B=1 synthesis;
  * without a vocoder checkpoint the Griffin-Lim fallback runs on the CPU (`tts_amd.audio`);
  * checkpoints load with `torch.load(..., weights_only=True)`;
  * sentence splitting and the text front end are the stand-ins of `tts_amd.text` (pysbd,
    phonemizer, unidecode and inflect are not in this image); phoneme configs need a
    `phonemize` callable;
  * several GPUs (config ``num_gpus`` > 1, or an explicit ``gpu_devices`` list): the sentences of a
    call are sharded over one worker process per GPU (`tts_amd.multigpu.GpuPool`, LPT on the
    token counts), each worker running this same batched path on its shard; results come back in
    sentence order. The workers start before this process touches the GPU.
"""
import functools
import json
import os
import time

import numpy as np
import torch

from .audio import AudioProcessor, wav_bytes
from .factories import load_config, setup_generator, setup_model
from .glow_tts import GlowTts
from .multigpu import GpuPool
from .vocoder import MultibandMelganGenerator
from .text import make_symbols, phonemes, split_into_sentences, symbols, text_to_seqvec


def _pool_synthesizer(config, phonemize, device):
    """GpuPool factory: a single-GPU Synthesizer on ``device`` inside a worker process."""
    torch.cuda.set_device(device)
    synth = Synthesizer(dict(config, num_gpus=1, gpu_devices=None), phonemize=phonemize)
    return synth.synthesize_batch


class Synthesizer:
    def __init__(self, config, phonemize=None):
        self.wavernn = None
        self.vocoder_model = None
        self.config = config
        self.phonemize = phonemize
        self.use_cuda = config["use_cuda"]
        self.pool = None
        devices = config.get("gpu_devices")
        if devices is None and int(config.get("num_gpus") or 1) > 1:
            devices = list(range(min(int(config["num_gpus"]), torch.cuda.device_count())))
        if self.use_cuda and devices is not None and len(devices) > 1:
            # one worker per GPU, started before this process makes any GPU call; every worker loads
            # the models, this process keeps the text front end and the audio processor only
            self.pool = GpuPool(functools.partial(_pool_synthesizer, dict(config), phonemize), devices)
            self.use_cuda = False
        if self.use_cuda:
            assert torch.cuda.is_available(), "CUDA is not availabe on this machine."
        self.tts_model = None
        if self.pool is not None:
            self.load_tts_config(config["tts_config"])
        else:
            self.load_tts(config["tts_checkpoint"], config["tts_config"], self.use_cuda)
            if config.get("vocoder_checkpoint"):
                self.load_vocoder(config["vocoder_checkpoint"], config["vocoder_config"], self.use_cuda)
        if config.get("wavernn_lib_path"):
            raise NotImplementedError("WaveRNN is outside the MI355X hot path (SURVEY.md §8f)")

    def load_tts_config(self, tts_config):
        """The config half of synthesizer.py:44-67: model config, audio processor, symbol tables,
        speaker mapping (what the text front end and the output stage need)."""
        self.tts_config = load_config(tts_config) if isinstance(tts_config, str) else tts_config
        self.use_phonemes = self.tts_config["use_phonemes"]
        self.ap = AudioProcessor(**self.tts_config["audio"])
        syms, phs = symbols, phonemes
        if "characters" in self.tts_config:
            syms, phs = make_symbols(**self.tts_config["characters"])
        self.input_size = len(phs) if self.use_phonemes else len(syms)
        # synthesizer.py:62-67: a speaker mapping (speakers.json, or a directory holding one) sets
        # num_speakers; tts(text, speaker_id) then conditions on the learned speaker table
        num_speakers = 0
        if self.config.get("tts_speakers") is not None:
            path = self.config["tts_speakers"]
            if os.path.splitext(path)[1] != ".json":
                path = os.path.join(path, "speakers.json")  # utils/speakers.py make_speakers_json_path
            try:
                with open(path) as f:
                    self.tts_speakers = json.load(f)
            except FileNotFoundError:
                self.tts_speakers = {}
            num_speakers = len(self.tts_speakers)
        self.num_speakers = num_speakers

    def load_tts(self, tts_checkpoint, tts_config, use_cuda):
        """synthesizer.py:44-82"""
        self.load_tts_config(tts_config)
        self.tts_model = setup_model(self.input_size, num_speakers=self.num_speakers, c=self.tts_config)
        cp = torch.load(tts_checkpoint, map_location=torch.device("cpu"), weights_only=True)
        self.tts_model.load_state_dict(cp["model"])
        if use_cuda:
            self.tts_model.cuda()
        self.tts_model.eval()
        if isinstance(self.tts_model, GlowTts):
            return
        # synthesizer.py:76 (3000); the optional config key ``max_decoder_steps`` overrides it
        self.tts_model.decoder.max_decoder_steps = int(self.config.get("max_decoder_steps") or 3000)
        if "r" in cp:
            self.tts_model.decoder.set_r(int(cp["r"]))
            print(f" > model reduction factor: {int(cp['r'])}")

    def load_vocoder(self, model_file, model_config, use_cuda):
        """synthesizer.py:84-94"""
        self.vocoder_config = load_config(model_config) if isinstance(model_config, str) else model_config
        self.vocoder_model = setup_generator(self.vocoder_config)
        self.vocoder_model.load_state_dict(torch.load(model_file, map_location="cpu", weights_only=True)["model"])
        self.vocoder_model.remove_weight_norm()
        self.vocoder_model.inference_padding = 0
        if use_cuda:
            self.vocoder_model.cuda()
        self.vocoder_model.eval()

    def save_wav(self, wav, path):
        self.ap.save_wav(np.array(wav), path)

    @staticmethod
    def split_into_sentences(text):
        return split_into_sentences(text)

    def synthesize_batch(self, sentences, speaker_id=None):
        """Sentences -> list of per-sentence waveforms (float32 numpy), one GPU call per model (per
        GPU when sharded over a pool)."""
        seqs = [text_to_seqvec(s, self.tts_config, self.phonemize) for s in sentences]
        if self.pool is not None:
            return self.pool.map(list(sentences), costs=[len(q) for q in seqs], speaker_id=speaker_id)
        lens = [max(1, len(q)) for q in seqs]
        dev = "cuda" if self.use_cuda else "cpu"
        batch = np.zeros((len(seqs), max(lens)), np.int64)
        for i, q in enumerate(seqs):
            batch[i, :len(q)] = q
        with torch.no_grad():
            wav = None
            if isinstance(self.tts_model, GlowTts):  # synthesis.py:60-66
                y = self.tts_model.inference(torch.from_numpy(batch).to(dev), lens)[0]
                post = y.transpose(1, 2)
                # a B = 1 reference call returns 2 * floor(y_length / 2) frames (decoder squeeze)
                mel_lens = [2 * (int(m) // 2) for m in self.tts_model.last_y_lengths]
            else:
                spk = None if speaker_id is None else torch.full((len(seqs),), int(speaker_id), dtype=torch.long)
                ids = torch.from_numpy(batch).to(dev)
                if isinstance(self.vocoder_model, MultibandMelganGenerator):
                    # both models in one library call (tts_taco_mbmelgan_infer), same waveforms
                    _, post, _, _, wav = self.tts_model.inference_vocoded(ids, self.vocoder_model, text_lengths=lens,
                                                                          speaker_ids=spk)
                else:
                    _, post, _, _ = self.tts_model.inference(ids, text_lengths=lens, speaker_ids=spk)
                mel_lens = [int(m) for m in self.tts_model.last_mel_lengths]
            if self.vocoder_model is not None:
                if wav is None:
                    wav = self.vocoder_model.inference(post.transpose(1, 2), lengths=mel_lens)
                hop = wav.shape[-1] // post.shape[1]
                wav = wav.reshape(len(seqs), -1).cpu().numpy()
                return [wav[i, :mel_lens[i] * hop] for i in range(len(seqs))]
        post = post.cpu().numpy()
        return [self.ap.inv_melspectrogram(post[i, :mel_lens[i]].T).astype(np.float32) for i in range(len(seqs))]

    def tts(self, text, speaker_id=None):
        """synthesizer.py:134-193"""
        start_time = time.time()
        sens = self.split_into_sentences(text)
        print(sens)
        wavs = []
        for wav in self.synthesize_batch(sens, speaker_id):
            wav = wav[:self.ap.find_endpoint(wav)]  # synthesis.py:130-131
            wavs += list(wav)
            wavs += [0] * 10000
        out = wav_bytes(self.ap, np.asarray(wavs, np.float32))
        process_time = time.time() - start_time
        audio_time = len(wavs) / self.tts_config["audio"]["sample_rate"]
        print(f" > Processing time: {process_time}")
        print(f" > Real-time factor: {process_time / audio_time}")
        return out

    def close(self):
        if self.pool is not None:
            self.pool.close()
            self.pool = None

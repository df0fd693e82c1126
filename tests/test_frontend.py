"""Synthesizer front end on the CPU: symbol tables (pinned against the reference), text cleaning,
sentence splitting, and the Griffin-Lim / trimming audio helpers (restated librosa pieces,
parity-unpinned: checked through their defining properties)."""
import io
import json
import os

import numpy as np
import scipy.io.wavfile

from tts_amd import text as T
from tts_amd.audio import AudioProcessor, mel_filterbank

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LJ_AUDIO = dict(fft_size=1024, win_length=1024, hop_length=256, sample_rate=22050, preemphasis=0.0,
                ref_level_db=20, power=1.5, griffin_lim_iters=30, num_mels=80, mel_fmin=50.0, mel_fmax=7600.0,
                spec_gain=1, signal_norm=True, min_level_db=-100, symmetric_norm=True, max_norm=4.0,
                clip_norm=True)


def test_symbol_tables_match_reference():
    g = json.load(open(os.path.join(GOLDEN, "text_symbols.json")))
    assert T.symbols == g["symbols"]
    assert T.phonemes == g["phonemes"]
    a = g["custom_make_symbols"]["args"]
    s, p = T.make_symbols(a[0], a[1], punctuations=a[2], pad=a[3], eos=a[4], bos=a[5])
    assert s == g["custom_make_symbols"]["symbols"] and p == g["custom_make_symbols"]["phonemes"]


def test_text_to_sequence_basic_and_arpabet():
    ids = T.text_to_sequence("Hello,   World!", ["basic_cleaners"])
    assert "".join(T.symbols[i] for i in ids) == "hello, world!"
    ids = T.text_to_sequence("Turn {HH AW1} left", ["basic_cleaners"])
    assert [T.symbols[i] for i in ids if T.symbols[i].startswith("@")] == []  # not in the default ARPAbet set
    s2i = {s: i for i, s in enumerate(T.symbols)}
    assert all(i not in (s2i["_"], s2i["~"], s2i["^"]) for i in ids)


def test_english_cleaners_numbers_and_abbreviations():
    c = T.english_cleaners
    assert c("Dr. Smith has 3 cats.") == "doctor smith has three cats."
    # replace_symbols runs after number expansion, so inflect's hyphens become spaces
    assert c("In 1984 it cost $5.50") == "in nineteen eighty four it cost five dollars, fifty cents"
    assert c("the 21st time") == "the twenty first time"
    assert T.number_to_words(1984, group=2, zero="oh") == "nineteen, eighty-four"
    assert T.number_to_words(1234567) == "one million, two hundred thirty-four thousand, five hundred sixty-seven"
    assert c("2,500 people & 2005 more") == "twenty five hundred people and two thousand five more"
    assert c("Café (open) 100") == "cafe open one hundred"


def test_sentence_split():
    assert T.split_into_sentences("Hello world.  How are you?  Fine!") == ["Hello world.", "How are you?", "Fine!"]
    assert T.split_into_sentences("no terminator") == ["no terminator"]


def test_mel_filterbank_slaney_properties():
    W = mel_filterbank(22050, 1024, 80, 50.0, 7600.0)
    assert W.shape == (80, 513) and (W >= 0).all()
    # Slaney normalisation: each triangle has unit area in Hz (up to bin quantisation)
    area = W.sum(1) * (22050 / 1024)
    assert np.all(np.abs(area[20:] - 1.0) < 0.05)
    # peaks are ordered and inside [fmin, fmax]
    peaks = W.argmax(1) * 22050 / 1024
    assert np.all(np.diff(peaks) >= 0) and peaks[0] >= 0 and peaks[-1] <= 7600 + 22050 / 1024


def test_stft_roundtrip_and_griffin_lim():
    ap = AudioProcessor(**LJ_AUDIO)
    rs = np.random.RandomState(0)
    t = np.arange(22050) / 22050.0
    y = 0.5 * np.sin(2 * np.pi * 220 * t) + 0.3 * np.sin(2 * np.pi * 1250 * t) + 0.01 * rs.randn(t.size)
    D = ap._stft(y)
    y2 = ap._istft(D)
    n = min(len(y), len(y2))
    assert np.abs(y[:n] - y2[:n]).max() < 1e-9
    mel = ap.melspectrogram(y)
    wav = ap.inv_melspectrogram(mel, rng=np.random.RandomState(1))
    mel2 = ap.melspectrogram(wav)
    m = min(mel.shape[1], mel2.shape[1])
    # GL reconstructs the magnitude envelope (phase is random): mel error well inside the range
    assert np.mean(np.abs(mel[:, :m] - mel2[:, :m])) < 0.35 * ap.max_norm


def test_find_endpoint_and_wav_bytes():
    ap = AudioProcessor(**LJ_AUDIO)
    wav = np.concatenate([0.5 * np.ones(30000), np.zeros(40000)])
    e = ap.find_endpoint(wav)
    assert 30000 <= e <= 30000 + 2 * int(22050 * 0.8 / 4)
    buf = io.BytesIO()
    ap.save_wav(wav, buf)
    sr, x = scipy.io.wavfile.read(io.BytesIO(buf.getvalue()))
    assert sr == 22050 and x.dtype == np.int16 and x.max() == 32767

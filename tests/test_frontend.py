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


def _write_stats(path, ap, wav, audio):
    """Stats as TTS/bin/compute_statistics.py:40-80 computes and saves them (np.save of a dict,
    range-normalisation keys removed from the stored audio config) for one waveform."""
    mel = ap.melspectrogram(wav)
    lin = ap.spectrogram(wav)
    n = mel.shape[1]
    mel_mean = mel.sum(1) / n
    lin_mean = lin.sum(1) / n
    stats = {"mel_mean": mel_mean, "mel_std": np.sqrt((mel ** 2).sum(1) / n - mel_mean ** 2),
             "linear_mean": lin_mean, "linear_std": np.sqrt((lin ** 2).sum(1) / n - lin_mean ** 2)}
    cfg = dict(audio, stats_path=str(path), signal_norm=True)
    for k in ("max_norm", "min_level_db", "symmetric_norm", "clip_norm"):
        del cfg[k]
    stats["audio_config"] = cfg
    np.save(path, stats, allow_pickle=True)
    return stats


def _test_wav():
    rs = np.random.RandomState(3)
    t = np.arange(2 * 22050) / 22050.0
    return 0.4 * np.sin(2 * np.pi * (180 + 300 * t) * t) + 0.2 * np.sin(2 * np.pi * 2100 * t) + 0.02 * rs.randn(t.size)


def test_mean_var_scaler_roundtrip(tmp_path):
    """tests/test_audio.py:157-176 (test_scaler): with `stats_path`, melspectrogram() is mean-var
    scaled and _denormalize() inverts it to the un-normalised mel within 1e-4; the stats file is the
    object array compute_statistics.py writes, computed here as compute_statistics.py does (the
    reference's own stats: test_reference_scale_stats_fixture_roundtrip)."""
    path = tmp_path / "scale_stats.npy"
    plain = AudioProcessor(**dict(LJ_AUDIO, signal_norm=False))
    wav = _test_wav()
    stats = _write_stats(path, plain, wav, LJ_AUDIO)
    ap = AudioProcessor(**dict(LJ_AUDIO, stats_path=str(path), do_trim_silence=True))
    assert ap.signal_norm is True and ap.max_norm is None and ap.symmetric_norm is None and ap.clip_norm is None
    mel_reference = plain.melspectrogram(wav)
    mel_norm = ap.melspectrogram(wav)
    assert np.allclose(mel_norm, (mel_reference - stats["mel_mean"][:, None]) / stats["mel_std"][:, None])
    assert abs(mel_norm.mean(1)).max() < 1e-6 and abs(mel_norm.std(1) - 1).max() < 1e-6
    mel_denorm = ap._denormalize(mel_norm)
    assert abs(mel_reference - mel_denorm).max() < 1e-4
    # the linear branch is selected by fft_size / 2 rows (audio.py:117), so the 513-row linear
    # spectrogram raises exactly as in the reference
    import pytest
    with pytest.raises(RuntimeError, match="Mean-Var stats"):
        ap.spectrogram(wav)
    # the stats were computed with other audio parameters: load_stats asserts (audio.py:174-179)
    with pytest.raises(AssertionError, match="mel_fmin"):
        AudioProcessor(**dict(LJ_AUDIO, mel_fmin=0.0, stats_path=str(path)))


def test_reference_scale_stats_fixture_roundtrip(tmp_path):
    """The reference's own mean-var stats (tests/inputs/scale_stats.npy, decoded statically into
    tests/golden/scale_stats_ref.npz by make_scale_stats.py: no unpickler runs on the reference
    file) through this AudioProcessor, as the reference's tests/test_audio.py:157-176 test_scaler
    runs them: its test_config.json audio section with preemphasis 0 and signal_norm, its
    example_1.wav; melspectrogram() then _denormalize() returns the un-normalised mel within 1e-4.
    load_stats' parameter check (audio.py:174-179) passes on the reference's stats_config, and the
    loader's .npy path (the object array compute_statistics.py writes, here written by this test
    from the fixture) returns the same stats as the .npz."""
    from tts_amd.audio import load_stats_file
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scale_stats_ref.npz")
    ref = load_stats_file(gold)
    with np.load(gold, allow_pickle=False) as z:
        test_audio = json.loads(str(z["test_audio"]))
        wav = z["wav_pcm16"].astype(np.float64) / 32768.0  # soundfile.read's float scaling
        sr = int(z["wav_sr"])
    assert ref["mel_mean"].shape == (80,) and ref["linear_std"].shape == (513,)
    assert ref["audio_config"]["num_mels"] == 80 and sr == test_audio["sample_rate"]
    # the .npy form of the same stats (this test's own file) through the restricted loader
    npy = tmp_path / "scale_stats.npy"
    np.save(npy, dict(ref), allow_pickle=True)
    again = load_stats_file(npy)
    for k in ("mel_mean", "mel_std", "linear_mean", "linear_std"):
        assert np.array_equal(again[k], ref[k])
    assert again["audio_config"] == ref["audio_config"]
    conf = dict(test_audio, preemphasis=0.0, do_trim_silence=True, signal_norm=True)
    ap = AudioProcessor(**dict(conf, stats_path=gold))
    plain = AudioProcessor(**dict(test_audio, preemphasis=0.0, signal_norm=False))
    mel_reference = plain.melspectrogram(wav)
    mel_norm = ap.melspectrogram(wav)
    assert np.allclose(mel_norm, (mel_reference - ref["mel_mean"][:, None]) / ref["mel_std"][:, None])
    mel_denorm = ap._denormalize(mel_norm)
    assert abs(mel_reference - mel_denorm).max() < 1e-4


def test_stats_loader_refuses_foreign_globals(tmp_path):
    """load_stats_file admits numpy array reconstruction and dicts only: a stats file whose pickle
    names any other callable is refused before that callable runs."""
    import pickle
    import pytest
    from tts_amd.audio import load_stats_file

    hit = tmp_path / "ran"

    class Evil:
        def __reduce__(self):
            return (open, (str(hit), "w"))

    arr = np.empty((), dtype=object)
    arr[()] = {"mel_mean": Evil()}
    path = tmp_path / "evil.npy"
    np.save(path, arr, allow_pickle=True)
    with pytest.raises(pickle.UnpicklingError, match="refused"):
        load_stats_file(path)
    assert not hit.exists()
    # the .npz form (audio_config as JSON) loads with allow_pickle=False
    npz = tmp_path / "stats.npz"
    np.savez(npz, mel_mean=np.zeros(80), mel_std=np.ones(80), linear_mean=np.zeros(513),
             linear_std=np.ones(513), audio_config=json.dumps({"num_mels": 80}))
    s = load_stats_file(npz)
    assert s["audio_config"] == {"num_mels": 80} and s["mel_std"].shape == (80,)

"""Host-side audio processing for Synthesizer.tts: the Griffin-Lim CPU fallback (config C1), silence
trimming and wav writing. Restates `TTS/utils/audio.py` (AudioProcessor) without librosa, which
is not in this image: the mel filterbank is librosa.filters.mel's published Slaney algorithm,
STFT/ISTFT are torch.stft/istft with librosa's conventions (periodic Hann, centred frames, the
config's pad mode), trimming is librosa.effects.trim's frame-RMS rule. Mean-var scaling (`stats_path`,
audio.py:80-86,108-186) reads compute_statistics.py's stats file through a restricted loader
(`load_stats_file`). None of these touch the GPU: the GPU path is the MB-MelGAN vocoder. Parity of the restated librosa pieces is unpinned
(librosa is not importable here to make fixtures); tests check their defining properties.
"""
import io
import json
import pickle

import numpy as np
import scipy.io.wavfile
import torch


def _hz_to_mel(f):
    """Slaney mel scale (librosa.hz_to_mel, htk=False)."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) with Slaney area normalisation."""
    fmax = sr / 2.0 if fmax is None else float(fmax)
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


class StandardScaler:
    """tts/utils/data.py:56-76."""

    def set_stats(self, mean, scale):
        self.mean_ = mean
        self.scale_ = scale

    def reset_stats(self):
        delattr(self, "mean_")
        delattr(self, "scale_")

    def transform(self, X):
        X = np.asarray(X)
        X -= self.mean_
        X /= self.scale_
        return X

    def inverse_transform(self, X):
        X = np.asarray(X)
        X *= self.scale_
        X += self.mean_
        return X


class _StatsConfig(dict):
    """Stand-in for `TTS.utils.io.AttrDict`, the class compute_statistics.py pickles the audio
    config as: keys as attributes, nothing else."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setstate__(self, state):  # the pickled __dict__ is the dict itself (AttrDict)
        pass


class _StatsUnpickler(pickle.Unpickler):
    """Admits exactly what `np.save(path, stats_dict)` writes: numpy array / dtype / scalar
    reconstruction, builtin containers, and the reference's AttrDict (as a plain dict). Any other
    global in the stream is refused before anything from it runs (the same rule as
    torch.load(weights_only=True))."""

    _NUMPY = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
              ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
              ("numpy", "ndarray"), ("numpy", "dtype")}

    def find_class(self, module, name):
        if (module, name) in self._NUMPY:
            return super().find_class(module, name)
        if name == "AttrDict" and module in ("TTS.utils.io", "mozilla_voice_tts.utils.io"):
            return _StatsConfig
        raise pickle.UnpicklingError(f"stats file references {module}.{name}: refused")


def load_stats_file(path):
    """The mean-var stats dict (mel_mean, mel_std, linear_mean, linear_std, audio_config).
    `.npz`: plain arrays (audio_config as a JSON string), read with allow_pickle=False. `.npy`:
    the object array compute_statistics.py writes (`np.save(path, dict, allow_pickle=True)`),
    read through `_StatsUnpickler` instead of numpy's unrestricted pickle load."""
    if str(path).endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            out = {k: z[k] for k in ("mel_mean", "mel_std", "linear_mean", "linear_std")}
            out["audio_config"] = json.loads(str(z["audio_config"]))
        return out
    with open(path, "rb") as f:
        version = np.lib.format.read_magic(f)
        read_header = (np.lib.format.read_array_header_1_0 if version == (1, 0)
                       else np.lib.format.read_array_header_2_0)
        _shape, _fortran, dtype = read_header(f)
        if not dtype.hasobject:
            raise ValueError(f"{path}: expected the pickled stats dict, found a plain {dtype} array")
        arr = _StatsUnpickler(f).load()
    stats = arr.item() if isinstance(arr, np.ndarray) else arr
    if not isinstance(stats, dict):
        raise ValueError(f"{path}: stats file does not hold a dict")
    return stats


class AudioProcessor:
    """The subset of TTS/utils/audio.py:11-345 that Synthesizer.tts uses."""

    def __init__(self, sample_rate=None, num_mels=None, min_level_db=None, frame_shift_ms=None,
                 frame_length_ms=None, hop_length=None, win_length=None, ref_level_db=None, fft_size=1024,
                 power=None, preemphasis=0.0, signal_norm=None, symmetric_norm=None, max_norm=None,
                 mel_fmin=None, mel_fmax=None, spec_gain=20, stft_pad_mode="reflect", clip_norm=True,
                 griffin_lim_iters=None, do_trim_silence=False, trim_db=60, stats_path=None, **_):
        self.sample_rate = sample_rate
        self.num_mels = num_mels
        self.min_level_db = min_level_db or 0
        self.ref_level_db = ref_level_db
        self.fft_size = fft_size
        self.power = power
        self.preemphasis = preemphasis
        self.griffin_lim_iters = griffin_lim_iters
        self.signal_norm = signal_norm
        self.symmetric_norm = symmetric_norm
        self.max_norm = 1.0 if max_norm is None else float(max_norm)
        self.mel_fmin = mel_fmin or 0
        self.mel_fmax = mel_fmax
        self.spec_gain = float(spec_gain)
        self.stft_pad_mode = stft_pad_mode
        self.clip_norm = clip_norm
        self.do_trim_silence = do_trim_silence
        self.trim_db = trim_db
        self.frame_shift_ms, self.frame_length_ms = frame_shift_ms, frame_length_ms
        self.do_sound_norm = _.get("do_sound_norm", False)
        self.stats_path = stats_path
        if hop_length is None:  # audio.py:99-105
            factor = frame_length_ms / frame_shift_ms
            assert float(factor).is_integer(), " [!] frame_shift_ms should divide frame_length_ms"
            hop_length = int(frame_shift_ms / 1000.0 * sample_rate)
            win_length = int(hop_length * factor)
        self.hop_length, self.win_length = hop_length, win_length
        assert self.min_level_db != 0.0, " [!] min_level_db is 0"
        assert self.win_length <= self.fft_size, " [!] win_length cannot be larger than fft_size"
        self.mel_basis = mel_filterbank(sample_rate, fft_size, num_mels, self.mel_fmin, self.mel_fmax)
        self.inv_mel_basis = np.linalg.pinv(self.mel_basis)
        if stats_path:  # audio.py:80-86: mean-var scaling replaces the range normalisation
            mel_mean, mel_std, linear_mean, linear_std, _cfg = self.load_stats(stats_path)
            self.setup_scaler(mel_mean, mel_std, linear_mean, linear_std)
            self.signal_norm = True
            self.max_norm = None
            self.clip_norm = None
            self.symmetric_norm = None

    # -- mean-var scaling (audio.py:165-186, tts/utils/data.py:56-76)
    def load_stats(self, stats_path):
        """audio.py:165-180: the stats file `TTS/bin/compute_statistics.py:59-80` writes, checked
        against this processor's parameters (the same skip list)."""
        stats = load_stats_file(stats_path)
        stats_config = stats["audio_config"]
        skip = ["griffin_lim_iters", "stats_path", "do_trim_silence", "ref_level_db", "power"]
        for key in stats_config.keys():
            if key in skip or key == "sample_rate":
                continue
            assert stats_config[key] == self.__dict__[key], \
                f" [!] Audio param {key} does not match the value used for computing mean-var stats. " \
                f"{stats_config[key]} vs {self.__dict__[key]}"
        return stats["mel_mean"], stats["mel_std"], stats["linear_mean"], stats["linear_std"], stats_config

    def setup_scaler(self, mel_mean, mel_std, linear_mean, linear_std):
        self.mel_scaler = StandardScaler()
        self.mel_scaler.set_stats(mel_mean, mel_std)
        self.linear_scaler = StandardScaler()
        self.linear_scaler.set_stats(linear_mean, linear_std)

    def _scaler_for(self, S):
        """audio.py:114-120 / 143-149: picked by the feature count. The linear branch compares
        with fft_size / 2 exactly as the reference does."""
        if S.shape[0] == self.num_mels:
            return self.mel_scaler
        if S.shape[0] == self.fft_size / 2:
            return self.linear_scaler
        raise RuntimeError(" [!] Mean-Var stats does not match the given feature dimensions.")

    # -- normalisation (audio.py:108-163)
    def _normalize(self, S):
        if not self.signal_norm:
            return S.copy()
        if hasattr(self, "mel_scaler"):
            return self._scaler_for(S).transform(S.copy().T).T
        S = S - self.ref_level_db
        S_norm = (S - self.min_level_db) / (-self.min_level_db)
        if self.symmetric_norm:
            S_norm = (2 * self.max_norm) * S_norm - self.max_norm
            return np.clip(S_norm, -self.max_norm, self.max_norm) if self.clip_norm else S_norm
        S_norm = self.max_norm * S_norm
        return np.clip(S_norm, 0, self.max_norm) if self.clip_norm else S_norm

    def _denormalize(self, S):
        S = S.copy()
        if not self.signal_norm:
            return S
        if hasattr(self, "mel_scaler"):
            return self._scaler_for(S).inverse_transform(S.T).T
        if self.symmetric_norm:
            if self.clip_norm:
                S = np.clip(S, -self.max_norm, self.max_norm)
            S = (S + self.max_norm) * -self.min_level_db / (2 * self.max_norm) + self.min_level_db
            return S + self.ref_level_db
        if self.clip_norm:
            S = np.clip(S, 0, self.max_norm)
        return S * -self.min_level_db / self.max_norm + self.min_level_db + self.ref_level_db

    def _amp_to_db(self, x):
        return self.spec_gain * np.log10(np.maximum(1e-5, x))

    def _db_to_amp(self, x):
        return np.power(10.0, x / self.spec_gain)

    # -- STFT (audio.py:259-279), librosa conventions on torch
    def _window(self):
        return torch.hann_window(self.win_length, periodic=True, dtype=torch.float64)

    def _stft(self, y):
        t = torch.as_tensor(np.asarray(y, np.float64))
        D = torch.stft(t, self.fft_size, self.hop_length, self.win_length, self._window(), center=True,
                       pad_mode=self.stft_pad_mode, return_complex=True)
        return D.numpy()

    def _istft(self, D):
        t = torch.as_tensor(D)
        return torch.istft(t, self.fft_size, self.hop_length, self.win_length, self._window(), center=True).numpy()

    def _griffin_lim(self, S, rng=None):
        rng = np.random if rng is None else rng
        angles = np.exp(2j * np.pi * rng.rand(*S.shape))
        S_complex = np.abs(S).astype(np.complex128)
        y = self._istft(S_complex * angles)
        for _ in range(self.griffin_lim_iters):
            angles = np.exp(1j * np.angle(self._stft(y)))
            y = self._istft(S_complex * angles)
        return y

    def _preemph_stft(self, y):
        if self.preemphasis != 0:  # audio.py:198-202
            import scipy.signal
            y = scipy.signal.lfilter([1, -self.preemphasis], [1], y)
        return self._stft(y)

    def spectrogram(self, y):
        """audio.py:216-222."""
        return self._normalize(self._amp_to_db(np.abs(self._preemph_stft(y))))

    def melspectrogram(self, y):
        """audio.py:224-230."""
        return self._normalize(self._amp_to_db(self.mel_basis @ np.abs(self._preemph_stft(y))))

    def inv_melspectrogram(self, mel, rng=None):
        """audio.py:241-248 (no pre-emphasis path: raise as the reference would need scipy lfilter)."""
        S = self._db_to_amp(self._denormalize(mel))
        S = np.maximum(1e-10, self.inv_mel_basis @ S)
        if self.preemphasis != 0:
            import scipy.signal
            return scipy.signal.lfilter([1], [1, -self.preemphasis], self._griffin_lim(S ** self.power, rng))
        return self._griffin_lim(S ** self.power, rng)

    # -- trimming / saving (audio.py:302-341)
    def find_endpoint(self, wav, threshold_db=-40, min_silence_sec=0.8):
        """audio.py:302-309: first window of min_silence_sec whose peak is below threshold_db."""
        window_length = int(self.sample_rate * min_silence_sec)
        hop_length = int(window_length / 4)
        threshold = self._db_to_amp(threshold_db)
        for x in range(hop_length, len(wav) - window_length, hop_length):
            if np.max(wav[x:x + window_length]) < threshold:
                return x + hop_length
        return len(wav)

    def trim_silence(self, wav):
        margin = int(self.sample_rate * 0.01)
        wav = wav[margin:-margin]
        n, hop, fl = len(wav), self.hop_length, self.win_length
        if n == 0:
            return wav
        yp = np.pad(wav, fl // 2, mode="reflect") if n > fl // 2 else np.pad(wav, fl // 2)
        nfr = 1 + (len(yp) - fl) // hop
        if nfr < 1:
            return wav
        idx = np.arange(fl)[None, :] + hop * np.arange(nfr)[:, None]
        mse = np.mean(np.abs(yp[idx]) ** 2, axis=1)
        db = 10.0 * np.log10(np.maximum(1e-10, mse)) - 10.0 * np.log10(np.maximum(1e-10, mse.max()))
        nz = np.flatnonzero(db > -self.trim_db)
        if nz.size == 0:
            return wav[:0]
        return wav[nz[0] * hop:min(n, (nz[-1] + 1) * hop)]

    def save_wav(self, wav, path):
        wav_norm = np.asarray(wav) * (32767 / max(0.01, np.max(np.abs(wav))))
        scipy.io.wavfile.write(path, self.sample_rate, wav_norm.astype(np.int16))


def wav_bytes(ap, wav):
    out = io.BytesIO()
    ap.save_wav(wav, out)
    return out

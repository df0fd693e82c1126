"""Host-side audio processing for Synthesizer.tts: the Griffin-Lim CPU fallback (config C1), silence
trimming and wav writing. Restates `TTS/utils/audio.py` (AudioProcessor) without librosa, which
is not in this image: the mel filterbank is librosa.filters.mel's published Slaney algorithm,
STFT/ISTFT are torch.stft/istft with librosa's conventions (periodic Hann, centred frames, the
config's pad mode), trimming is librosa.effects.trim's frame-RMS rule. None of these touch the
GPU: the GPU path is the MB-MelGAN vocoder. Parity of the restated librosa pieces is unpinned
(librosa is not importable here to make fixtures); tests check their defining properties.
"""
import io

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
        if stats_path:
            raise NotImplementedError("mean-var stats (stats_path) are not restated in this build")
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

    # -- normalisation (audio.py:108-163)
    def _normalize(self, S):
        if not self.signal_norm:
            return S.copy()
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

    def melspectrogram(self, y):
        D = self._stft(y)
        return self._normalize(self._amp_to_db(self.mel_basis @ np.abs(D)))

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

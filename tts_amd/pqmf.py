"""PQMF filter-bank coefficients (host, load time).

Restates ``TTS/vocoder/layers/pqmf.py:10-43``: a Kaiser-windowed FIR prototype from
``scipy.signal.firwin(taps + 1, cutoff, window=('kaiser', beta))`` (pinned third-party
algorithm, scipy present in this image), cosine-modulated into analysis ``H`` and
synthesis ``G`` banks, with the reference's ``(taps - 1) / 2`` phase centre kept as is
(``pqmf.py:25``), computed in float64 and cast to float32 like ``torch.from_numpy(...).float()``.
"""

import numpy as np


def pqmf_filters(N: int = 4, taps: int = 62, cutoff: float = 0.15, beta: float = 9.0):
    from scipy import signal as sig
    qmf = sig.firwin(taps + 1, cutoff, window=("kaiser", beta))
    H = np.zeros((N, taps + 1))
    G = np.zeros((N, taps + 1))
    n = np.arange(taps + 1)
    for k in range(N):
        cf = (2 * k + 1) * (np.pi / (2 * N)) * (n - (taps - 1) / 2)
        ph = (-1) ** k * np.pi / 4
        H[k] = 2 * qmf * np.cos(cf + ph)
        G[k] = 2 * qmf * np.cos(cf - ph)
    updown = np.zeros((N, N, N), dtype=np.float32)
    for k in range(N):
        updown[k, k, 0] = 1.0
    return (H[:, None, :].astype(np.float32), G[None, :, :].astype(np.float32), updown)

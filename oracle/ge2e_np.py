"""ORACLE (test infrastructure only): float32 numpy restatement of the reference GE2E speaker
encoder (``TTS/speaker_encoder/model.py``). Only ``tests/`` may import it.

Parity pin: ``tests/golden/ge2e.npz`` was produced by running the reference in the build container
(``tests/golden/make_golden.py ge2e``).

* ``model.py:5-17``   LSTMWithProjection: nn.LSTM(in -> H) over the sequence, then Linear(H -> P)
* ``model.py:19-30``  LSTMWithoutProjection: num_layers-deep nn.LSTM, relu(Linear(h_n[-1]))
* ``model.py:62-68``  inference: last frame, F.normalize(p=2, dim=1)
* ``model.py:70-88``  compute_embedding: mean over windows of num_frames, hop num_frames - overlap
"""

import numpy as np

F32 = np.float32


def _sig(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x.astype(F32)))).astype(F32)


def lstm_seq(x, w_ih, w_hh, b_ih, b_hh):
    """torch.nn.LSTM (one layer, batch_first, zero initial state) on x (T, D) -> (T, H)."""
    H = w_hh.shape[1]
    xin = (x @ w_ih.T + b_ih).astype(F32)
    h = np.zeros(H, F32)
    c = np.zeros(H, F32)
    out = np.zeros((x.shape[0], H), F32)
    for t in range(x.shape[0]):
        g = xin[t] + (h @ w_hh.T + b_hh)
        i, f = _sig(g[:H]), _sig(g[H:2 * H])
        gg, o = np.tanh(g[2 * H:3 * H]).astype(F32), _sig(g[3 * H:])
        c = (f * c + i * gg).astype(F32)
        h = (o * np.tanh(c)).astype(F32)
        out[t] = h
    return out


class Ge2eOracle:
    def __init__(self, sd, num_layers=3, with_proj=True):
        self.sd = {k: np.asarray(v, F32) for k, v in sd.items()}
        self.nl = num_layers
        self.with_proj = with_proj

    def inference(self, x):
        """one sequence x (T, D) -> (P,)"""
        sd = self.sd
        y = np.asarray(x, F32)
        if self.with_proj:
            for i in range(self.nl):
                p = f"layers.{i}.lstm."
                o = lstm_seq(y, sd[p + "weight_ih_l0"], sd[p + "weight_hh_l0"], sd[p + "bias_ih_l0"], sd[p + "bias_hh_l0"])
                y = (o @ sd[f"layers.{i}.linear.weight"].T).astype(F32)
            d = y[-1]
        else:
            for k in range(self.nl):
                p = "layers.lstm."
                y = lstm_seq(y, sd[p + f"weight_ih_l{k}"], sd[p + f"weight_hh_l{k}"], sd[p + f"bias_ih_l{k}"],
                             sd[p + f"bias_hh_l{k}"])
            d = np.maximum(y[-1] @ sd["layers.linear.weight"].T + sd["layers.linear.bias"], F32(0)).astype(F32)
        n = max(float(np.sqrt((d.astype(np.float64) ** 2).sum())), 1e-12)
        return (d / F32(n)).astype(F32)

    def compute_embedding(self, x, num_frames=160, overlap=0.5):
        x = np.asarray(x, F32)
        hop = num_frames - int(num_frames * overlap)
        embs = [self.inference(x[o:min(len(x), o + num_frames)]) for o in range(0, len(x), hop)]
        return (np.sum(embs, axis=0) / F32(len(embs))).astype(F32)

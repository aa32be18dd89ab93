"""The oracle's dropout-mask restatement (oracle/savqa_oracle.py:dropout_keep) against a
scalar pure-Python statement of the stream documented in include/savqa.h, plus its
statistics (keep rate 1-p, independence across sites and seeds)."""
import numpy as np

from oracle import savqa_oracle as O

M64 = (1 << 64) - 1


def splitmix_bits(seed, site, idx):
    z = (seed + site * 0xD1B54A32D192ED03 + (idx + 1) * 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z >> 32


def test_keep_matches_scalar_statement():
    for seed, site, p in ((0, 1, 0.5), (2 ** 63 - 5, 8, 0.1), (123456789, 4, 0.9)):
        k = O.dropout_keep(seed, site, 300, p)
        thr = int(p * 2 ** 32)
        ref = np.array([splitmix_bits(seed, site, i) >= thr for i in range(300)])
        assert (k == ref).all()


def test_keep_statistics():
    n = 1 << 20
    for p in (0.1, 0.5, 0.9):
        k = O.dropout_keep(42, 2, n, p)
        assert abs(k.mean() - (1 - p)) < 4 / np.sqrt(n)
    a, b = O.dropout_keep(42, 2, n, 0.5), O.dropout_keep(42, 3, n, 0.5)
    c = O.dropout_keep(43, 2, n, 0.5)
    for x in (b, c):
        assert abs((a == x).mean() - 0.5) < 4 / np.sqrt(n)
    assert O.dropout_keep(1, 1, 64, 0.0).all() and not O.dropout_keep(1, 1, 64, 1.0).any()


def test_oracle_dropout_identity_when_off():
    import torch
    x = torch.randn(4, 5)
    assert torch.equal(O.dropout(x, None, 2), x)
    assert torch.equal(O.dropout(x, (7, 0.5), -1), x)
    y = O.dropout(x, (7, 0.5), 2)
    kept = y != 0
    assert torch.allclose(y[kept], 2 * x[kept])

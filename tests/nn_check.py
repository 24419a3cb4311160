"""Helpers for the network numerics tests.

The only floating-point parity in the system is the value/policy network: the search is
exact given its values.  A check therefore has to be able to FAIL on a broken head, so every
comparison here asserts two things:

* max |got - want| <= atol, with atol a small fraction of the outputs' spread (`spread_ok`
  refuses a comparison whose reference outputs barely vary), and
* the Pearson correlation of got and want >= min_r (a near-constant head fails it even when
  the outputs sit inside a loose band).

`fp16_emulation` restates the GPU path's numerics on the CPU in float64: BN folded, weights
rounded to fp16, every layer's activation rounded to fp16 (the tower's epilogue stores fp16),
accumulation exact.  It predicts the fp16-vs-fp32 error a correct kernel must show.
"""
import numpy as np
import torch


def pearson(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    a = a - a.mean()
    b = b - b.mean()
    return float((a @ b) / np.sqrt((a @ a) * (b @ b)))


def assert_tracks(got, want, atol, min_r=0.999, min_std=None, what=""):
    got = np.asarray(got, np.float64).reshape(-1)
    want = np.asarray(want, np.float64).reshape(-1)
    assert got.shape == want.shape, what
    err = float(np.abs(got - want).max())
    assert err <= atol, f"{what}: max |err| {err:.3e} > atol {atol:.1e}"
    if min_std is not None:
        assert want.std() >= min_std, f"{what}: reference outputs span too little ({want.std():.3e})"
    if len(want) > 2:
        r = pearson(got, want)
        assert r >= min_r, f"{what}: Pearson {r:.6f} < {min_r}"
    return err


def fails_tracking(got, want, atol, min_r=0.999) -> bool:
    """True when `assert_tracks` would reject got (the mutation checks: a broken head)."""
    try:
        assert_tracks(got, want, atol, min_r)
    except AssertionError:
        return True
    return False


def fp16_emulation_features(folded, x):
    """Pooled tower features [n, 128] of a FoldedValueNetwork under the GPU path's fp16
    storage points (float64 accumulation)."""
    def h(t):
        return t.half().double()

    def conv(c, t):
        return torch.nn.functional.conv2d(t, h(c.weight.double()), c.bias.double(), padding=1)

    with torch.no_grad():
        a = h(torch.relu(conv(folded.stem, x.double())))
        for b in folded.res:
            t = h(torch.relu(conv(b.c1, a)))
            a = h(torch.relu(a + conv(b.c2, t)))
        return a.mean(dim=(2, 3))


def features64(folded, x):
    with torch.no_grad():
        f = folded.double()
        a = torch.relu(f.stem(x.double()))
        for b in f.res:
            a = torch.relu(a + b.c2(torch.relu(b.c1(a))))
        return a.mean(dim=(2, 3))


def wide_head(features, std=1.2):
    """(weight [128], bias) of a Linear head along the top principal direction of `features`
    [n, 128], scaled so the pre-tanh sum has mean 0 and std `std` over these inputs."""
    f = features.double()
    mu = f.mean(0)
    _, _, vt = torch.linalg.svd(f - mu, full_matrices=False)
    d = vt[0]
    scale = std / ((f - mu) @ d).std().item()
    return (d * scale).float(), float(-(mu @ (d * scale)).item())

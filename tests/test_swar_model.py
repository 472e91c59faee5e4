"""CPU model of the SWAR tile kernel's horizontal arithmetic
(kernels/swar_device.hpp ``horiz``): the pair-sum form

    P_j = X_j + X_{j+CH},   H_k = P_{k-CH} + P_k

over one 64-lane strip, the operands past a lane's last / before its first
word read from the neighbouring lane (DPP wave_shl / wave_shr, 0 past the
wave edge).  At lane 0 it differs from the direct form 2 X_k + X_{k-CH} +
X_{k+CH} (both terms of P_{k-CH} are missing there instead of one); the
kernel's halo of ceil(steps * CH / LW) lanes per side must still absorb what
enters from the strip edges.  Checked here for every lane width, channel
count and step count the kernels use, against the reference oracle
(``numpy_convolve``): the kept lanes are exact, and the two forms differ only
inside the halo.
"""
import numpy as np
import pytest


def _strip_steps(img, x0, lw, ch, steps, pair_sums):
    """Run `steps` gaussian repetitions on the 64-lane strip starting at byte
    x0 of every row (whole image height: the vertical direction is exact), the
    strip's outside treated as unknown (0 past the wave edge), columns outside
    the image re-zeroed every step.  Returns the strip's bytes [rows, 64*lw]."""
    rows, width = img.shape
    pos = x0 + np.arange(64 * lw)
    inside = (pos >= 0) & (pos < width)
    x = np.zeros((rows, 64 * lw), np.int64)
    x[:, inside] = img[:, pos[inside]]
    for _ in range(steps):
        X = x.reshape(rows, 64, lw)
        if pair_sums:
            P = np.zeros_like(X)
            for j in range(lw):
                if j + ch < lw:
                    P[:, :, j] = X[:, :, j] + X[:, :, j + ch]
                else:  # X_{j+CH} from lane + 1 (wave_shl:1; 0 past lane 63)
                    nb = np.zeros_like(X[:, :, 0])
                    nb[:, :-1] = X[:, 1:, j + ch - lw]
                    P[:, :, j] = X[:, :, j] + nb
            H = np.zeros_like(X)
            for k in range(lw):
                if k >= ch:
                    H[:, :, k] = P[:, :, k - ch] + P[:, :, k]
                else:  # P_{k-CH} from lane - 1 (wave_shr:1; 0 before lane 0)
                    nb = np.zeros_like(P[:, :, 0])
                    nb[:, 1:] = P[:, :-1, k - ch + lw]
                    H[:, :, k] = nb + P[:, :, k]
        else:
            flat = X.reshape(rows, -1)
            left = np.zeros_like(flat)
            right = np.zeros_like(flat)
            left[:, ch:] = flat[:, :-ch]
            right[:, :-ch] = flat[:, ch:]
            H = (2 * flat + left + right).reshape(rows, 64, lw)
        h = H.reshape(rows, -1)
        up = np.zeros_like(h)
        dn = np.zeros_like(h)
        up[1:] = h[:-1]
        dn[:-1] = h[1:]
        x = (up + 2 * h + dn) >> 4  # floor(S / 16), every sum < 4080
        x[:, ~inside] = 0
    return x


@pytest.mark.parametrize("lw", [4, 8])
@pytest.mark.parametrize("ch", [1, 3, 4])
def test_pair_sum_horizontal_keeps_halo_contract(pconv_mod, rng, lw, ch):
    if ch > lw:
        return
    rows = 13
    width = 64 * lw * 3 + 37
    img = rng.integers(0, 256, size=(rows, width), dtype=np.uint8)
    max_steps = (32 * lw - 1) // ch  # halo lanes per side must stay < 32
    for steps in sorted({1, 2, 3, min(8, max_steps), min(12, max_steps), max_steps}):
        hl = (steps * ch + lw - 1) // lw
        # the reference on a grey frame of `width` bytes: the kernels treat a
        # row as bytes with tap distance CH, i.e. CH interleaved grey images
        ref = np.empty((rows, width), np.int64)
        for c in range(ch):
            ref[:, c::ch] = pconv_mod.numpy_convolve(np.ascontiguousarray(img[:, c::ch]), steps, "gaussian")
        for x0 in (-hl * lw, 64 * lw - 2 * hl * lw + 5, width - 64 * lw + hl * lw):  # left edge, interior, right edge
            got = _strip_steps(img, x0, lw, ch, steps, pair_sums=True)
            direct = _strip_steps(img, x0, lw, ch, steps, pair_sums=False)
            kept = slice(hl * lw, (64 - hl) * lw)
            pos = x0 + np.arange(64 * lw)[kept]
            ok = (pos >= 0) & (pos < width)
            assert np.array_equal(got[:, kept][:, ok], ref[:, pos[ok]]), (lw, ch, steps, x0)
            assert np.array_equal(got[:, kept], direct[:, kept]), (lw, ch, steps, x0)
            # the forms may differ only inside the halo
            diff = np.nonzero((got != direct).any(axis=0))[0]
            assert np.all((diff < hl * lw) | (diff >= (64 - hl) * lw)), (lw, ch, steps, x0)

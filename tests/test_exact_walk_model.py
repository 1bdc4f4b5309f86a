"""CPU model of the exact descriptor kernel's bin ownership
(descriptor.hip k_descriptor_exact): per 64-sample chunk, each sample's
trilinear contributions are rearranged per target cell into {P, S} records,
and lane (cell, orientation pair g) walks its samples in ascending order
adding P to bins (2g, 2g+1) when it is the sample's primary owner
(g == o0 >> 1) and S to bins (2g, 8) otherwise.  The resulting float32 bins
must equal OpenCV's sequential per-sample accumulation (calcSIFTDescriptor:
hist[idx + ...] += v_rco...) bit for bit, including the +0 adds."""
import numpy as np

D, NB = 4, 8


def opencv_hist(samples):
    """calcSIFTDescriptor's histogram: (d+2)^2 cells x (n+2) slots, float32, raster order."""
    hist = np.zeros(((D + 2) * (D + 2), NB + 2), np.float32)
    for r0, c0, o0, v in samples:
        for dr in (0, 1):
            for dc in (0, 1):
                cell = (r0 + 1 + dr) * (D + 2) + (c0 + 1 + dc)
                for do in (0, 1):
                    hist[cell, o0 + do] = np.float32(hist[cell, o0 + do] + v[dr * 4 + dc * 2 + do])
    out = np.zeros((D * D, NB), np.float32)
    for i in range(D):
        for j in range(D):
            h = hist[(i + 1) * (D + 2) + (j + 1)]
            out[i * D + j] = h[:NB]
            out[i * D + j, 0] = np.float32(h[0] + h[NB])
            out[i * D + j, 1] = np.float32(h[1] + h[NB + 1])
    return out


def kernel_hist(samples):
    """The owner-lane walk over {P, S} records, chunk by chunk."""
    acc = np.zeros((D * D, 4, 3), np.float32)  # (cell, g) -> A (bin 2g), B (bin 2g+1), W (bin 8)
    for k0 in range(0, len(samples), 64):
        chunk = samples[k0:k0 + 64]
        recs = []
        for r0, c0, o0, v in chunk:
            odd, seven = o0 & 1, o0 == NB - 1
            rec = {}
            for q in range(4):
                x, y = v[2 * q], v[2 * q + 1]
                rec[q] = (np.float32(0) if odd else x, x if odd else y,
                          y if (odd and not seven) else np.float32(0), y if seven else np.float32(0))
            recs.append((r0, c0, o0, rec))
        for cell in range(D * D):
            ci, cj = divmod(cell, D)
            for g in range(4):
                A, B, W = acc[cell, g]
                for r0, c0, o0, rec in recs:  # ascending sample order
                    if r0 not in (ci - 1, ci) or c0 not in (cj - 1, cj):
                        continue
                    if (o0 - 2 * g + 1) % NB >= 3:  # o0 in {2g - 1 mod 8, 2g, 2g + 1}
                        continue
                    p = rec[(ci - r0) * 2 + (cj - c0)]
                    prim = (o0 >> 1) == g
                    A = np.float32(A + (p[0] if prim else p[2]))
                    B = np.float32(B + (p[1] if prim else np.float32(0)))
                    W = np.float32(W + (np.float32(0) if prim else p[3]))
                acc[cell, g] = (A, B, W)
    out = np.zeros((D * D, NB), np.float32)
    for cell in range(D * D):
        for g in range(4):
            A, B, W = acc[cell, g]
            out[cell, 2 * g] = np.float32(A + W) if g == 0 else A
            out[cell, 2 * g + 1] = B
    return out


def random_samples(rng, n):
    s = []
    for _ in range(n):
        r0, c0, o0 = int(rng.integers(-1, D)), int(rng.integers(-1, D)), int(rng.integers(0, NB))
        mag = np.float32(rng.uniform(0, 50))
        rb, cb, ob = (np.float32(rng.uniform(0, 1)) for _ in range(3))
        # OpenCV's trilinear split (v_rco000 .. v_rco111), float32
        v_r1 = np.float32(mag * rb); v_r0 = np.float32(mag - v_r1)
        v_rc11 = np.float32(v_r1 * cb); v_rc10 = np.float32(v_r1 - v_rc11)
        v_rc01 = np.float32(v_r0 * cb); v_rc00 = np.float32(v_r0 - v_rc01)
        v = []
        for t in (v_rc00, v_rc01, v_rc10, v_rc11):
            hi = np.float32(t * ob)
            v += [np.float32(t - hi), hi]
        s.append((r0, c0, o0, v))
    return s


def test_owner_walk_equals_sequential_histogram():
    rng = np.random.default_rng(7)
    for n in (1, 63, 64, 65, 300):
        samples = random_samples(rng, n)
        a, b = opencv_hist(samples), kernel_hist(samples)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), n


def test_concentrated_orientation_band():
    """A raster chunk's thin band: every sample in two cell rows and near the
    dominant orientation (bins 7, 0, 1), the case that loads one lane most."""
    rng = np.random.default_rng(11)
    samples = random_samples(rng, 200)
    samples = [(1 + (i % 2) - 1, c0, (7, 0, 1)[i % 3], v) for i, (r0, c0, o0, v) in enumerate(samples)]
    assert np.array_equal(opencv_hist(samples).view(np.uint32), kernel_hist(samples).view(np.uint32))

"""CPU restatement of MultiModalX's noise augmentations — TEST INFRASTRUCTURE ONLY.

The checker for vitcnn_amd.window.PatchBatcher's radiation / mixture noise (SURVEY.md section 8 row
F2, next-row "radiation/mixture noise"); imported by tests/ and nothing else.  Restates
datasets.py:529-545 (radiation_noise, mixture_noise) as applied at datasets.py:565-568 to the HSI
patch after flip / rot90, given the per-sample decisions the batcher drew on the host and the
device's counter-based per-element randomness (restated here from patches.hip: splitmix64 over
(seed, sample id, stream, element), Box-Muller on two 24-bit uniforms).  The reference's own
randomness is numpy's global stream (np.random.normal / np.random.choice); the device draws these
fields from the hash instead, so the check is exact given the draws plus distributional
(tests/test_window_gpu.py): parity of the noise FIELDS with the reference is unpinned by design.

  radiation (datasets.py:529-532):  x' = alpha * x + beta * N,            beta = 1/25
  mixture   (datasets.py:534-545):  x' = (a1 * x + a2 * d2) / (a1 + a2) + beta * N
            d2[i, j, :] = data[indices[l]] for label[i, j] not ignored, l uniform over the positions
            with labels[l] == label[i, j] (labels unshuffled, indices shuffled: :505-506), else 0.
"""
import numpy as np

M64 = (1 << 64) - 1


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def noise_key(seed, gid, stream):
    return mix64(seed ^ mix64(((gid << 2) | stream) & M64))


def gauss(key, e):
    r = mix64((key + e) & M64)
    u1 = (float(r >> 40) + 0.5) / 16777216.0
    u2 = (float(r & 0xFFFFFF) + 0.5) / 16777216.0
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def apply_noise(x, lab, rad, mix, off, pix, cube, seed, gid0):
    """x [n, C, P, P] (float64 copy returned), lab [n, P, P] label windows, rad [n], mix [n, 2],
    off / pix the class -> source-pixel CSR, cube [W * H, C]."""
    x = np.array(x, dtype=np.float64)
    n, C, P, _ = x.shape
    PP = P * P
    nlab = len(off) - 1
    for s in range(n):
        a, (a1, a2) = float(rad[s]), (float(mix[s, 0]), float(mix[s, 1]))
        gid = gid0 + s
        if a == 0.0 and not a1 > 0.0:
            continue
        xs = x[s].reshape(C, PP)
        if a != 0.0:
            k0 = noise_key(seed, gid, 0)
            for c in range(C):
                for p in range(PP):
                    xs[c, p] = a * xs[c, p] + 0.04 * gauss(k0, c * PP + p)
        if a1 > 0.0:
            k1, k2 = noise_key(seed, gid, 1), noise_key(seed, gid, 2)
            d2 = np.zeros((C, PP))
            labs = np.asarray(lab[s]).reshape(PP)
            for p in range(PP):
                lv = int(labs[p])
                if 0 <= lv < nlab and off[lv + 1] > off[lv]:
                    cnt = int(off[lv + 1] - off[lv])
                    j = (mix64((k2 + p) & M64) >> 32) % cnt
                    d2[:, p] = cube[int(pix[off[lv] + j])]
            for c in range(C):
                for p in range(PP):
                    xs[c, p] = (a1 * xs[c, p] + a2 * d2[c, p]) / (a1 + a2) + 0.04 * gauss(k1, c * PP + p)
        x[s] = xs.reshape(C, P, P)
    return x

"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

Numpy restatement of the training-augmentation members that s3od_amd/csrc/data_ops.hip builds on
device, following the published algorithms of the libraries the reference calls
(synth_sod/src/synth_sod/model_training/transforms.py:12-224 -> albumentations 2.0.8 / OpenCV 4.12,
pinned in /root/reference/uv.lock:249-251, 2875-2877).  Neither library is installed here, so parity
with them is UNPINNED: these functions pin the device kernels to the published algorithms as restated
below, on float images in [0, 1] (the reference runs them on uint8; 8-bit quantisation is restated
where the algorithm itself works on 8-bit values: CLAHE's L channel, JPEG samples, posterize).

Every function works on x: float [3, S, S] (RGB planes) unless stated otherwise.
"""
from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF


# ------------------------------------------------------------------ counter-based RNG (data_ops.hip hash3)
def hash3(a, b, c):
    a = np.asarray(a, np.uint64); b = np.asarray(b, np.uint64); c = np.asarray(c, np.uint64)
    h = ((a * 0x9E3779B1) & M32) ^ (((b + 0x7F4A7C15) & M32) * 0x85EBCA77 & M32) ^ (((c + 0x165667B1) & M32) * 0xC2B2AE3D & M32)
    h = h & M32
    h ^= h >> 15; h = (h * 0x2C1B3C6D) & M32
    h ^= h >> 12; h = (h * 0x297A2D39) & M32
    h ^= h >> 15
    return h


def gauss(seed, pix, c):
    """Box-Muller standard normal of (seed, pixel, channel) (data_ops.hip gauss)."""
    h1, h2 = hash3(seed, pix, 2 * c), hash3(seed, pix, 2 * c + 1)
    u1 = ((h1 >> 8) + 1).astype(np.float32) * np.float32(1.0 / 16777217.0)
    u2 = (h2 >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return np.sqrt(-2.0 * np.log(u1.astype(np.float64))) * np.cos(2 * np.pi * u2.astype(np.float64))


def uni(seed, pix, c):
    return ((hash3(seed, pix, c) >> 8).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)


def poisson_inv(lam, u):
    """Poisson(lam) by sequential inversion of the uniform u (float32 recurrences, as the kernel)."""
    lam = np.float32(lam)
    p = np.full(u.shape, np.exp(-lam, dtype=np.float32), np.float32)
    F = p.copy()
    k = np.zeros(u.shape, np.int64)
    cap = int(3.0 * float(lam)) + 40
    for kk in range(1, cap + 1):
        act = u > F
        if not act.any():
            break
        p = np.where(act, (p * lam) / np.float32(kk), p).astype(np.float32)
        F = np.where(act, F + p, F).astype(np.float32)
        k = np.where(act, kk, k)
    return k


def reflect101(i, n):
    i = np.asarray(i)
    if n == 1:
        return np.zeros_like(i)
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)


# ------------------------------------------------------------------ colour spaces (cv2 float formulas)
def rgb2hls(x):
    """cv2 COLOR_RGB2HLS on float images: H degrees, L, S in [0, 1]."""
    r, g, b = x
    vmax, vmin = np.maximum(r, np.maximum(g, b)), np.minimum(r, np.minimum(g, b))
    diff = vmax - vmin
    l = (vmax + vmin) * 0.5
    ok = diff > 1.1920929e-7
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.where(l < 0.5, diff / (vmax + vmin), diff / (2.0 - vmax - vmin))
        k = 60.0 / diff
        h = np.where(vmax == r, (g - b) * k, np.where(vmax == g, (b - r) * k + 120.0, (r - g) * k + 240.0))
    h = np.where(h < 0, h + 360.0, h)
    return np.where(ok, h, 0.0), l, np.where(ok, s, 0.0)


_SECTOR = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])


def hls2rgb(h, l, s):
    p2 = np.where(l <= 0.5, l * (1 + s), l + s - l * s)
    p1 = 2 * l - p2
    hh = np.mod(h / 60.0, 6.0)
    sector = np.floor(hh).astype(int) % 6
    f = hh - np.floor(hh)
    tab = np.stack([p2, p1, p1 + (p2 - p1) * (1 - f), p1 + (p2 - p1) * f])
    idx = _SECTOR[sector]                                   # [..., 3]: b, g, r table indices
    pick = lambda j: np.take_along_axis(tab, idx[..., j][None], 0)[0]
    b, g, r = pick(0), pick(1), pick(2)
    grey = s == 0
    return np.stack([np.where(grey, l, r), np.where(grey, l, g), np.where(grey, l, b)])


def _lin(v):
    return np.where(v > 0.04045, ((v + 0.055) / 1.055) ** 2.4, v / 12.92)


def _srgb(v):
    return np.where(v > 0.0031308, 1.055 * np.maximum(v, 0) ** (1 / 2.4) - 0.055, 12.92 * v)


def _lab_f(t):
    return np.where(t > 0.008856, np.cbrt(t), 7.787 * t + 16.0 / 116.0)


def rgb2lab(x):
    r, g, b = _lin(x[0]), _lin(x[1]), _lin(x[2])
    X = (0.412453 * r + 0.357580 * g + 0.180423 * b) / 0.950456
    Y = 0.212671 * r + 0.715160 * g + 0.072169 * b
    Z = (0.019334 * r + 0.119193 * g + 0.950227 * b) / 1.088754
    fx, fy, fz = _lab_f(X), _lab_f(Y), _lab_f(Z)
    L = np.where(Y > 0.008856, 116.0 * fy - 16.0, 903.3 * Y)
    return L, 500.0 * (fx - fy), 200.0 * (fy - fz)


def lab2rgb(L, A, B):
    Y = np.where(L <= 8.0, L / 903.3, ((L + 16.0) / 116.0) ** 3)
    fy = np.where(L <= 8.0, 7.787 * Y + 16.0 / 116.0, (L + 16.0) / 116.0)
    fx, fz = A / 500.0 + fy, fy - B / 200.0
    X = np.where(fx > 0.206893, fx ** 3, (fx - 16.0 / 116.0) / 7.787) * 0.950456
    Z = np.where(fz > 0.206893, fz ** 3, (fz - 16.0 / 116.0) / 7.787) * 1.088754
    r = 3.240479 * X - 1.53715 * Y - 0.498535 * Z
    g = -0.969256 * X + 1.875991 * Y + 0.041556 * Z
    b = 0.055648 * X - 0.204043 * Y + 1.057311 * Z
    return np.clip(np.stack([_srgb(r), _srgb(g), _srgb(b)]), 0, 1)


# ------------------------------------------------------------------ group 1: CLAHE
def clahe(x, clip, tiles=8):
    """fpixel.clahe: cv2.createCLAHE(clipLimit, (8, 8)).apply on L of Lab (8-bit L = L*255/100), with
    cv2's CLAHE_CalcLut_Body (clip, redistribute batch + residual steps, rounded LUT) and
    CLAHE_Interpolation_Body (bilinear between the 4 nearest tile LUTs)."""
    S = x.shape[1]
    T = S // tiles
    L, A, B = rgb2lab(x)
    v = np.clip(np.rint(L * (255.0 / 100.0)), 0, 255).astype(int)
    area = T * T
    limit = max(int(clip * area / 256), 1)
    lut = np.zeros((tiles, tiles, 256))
    for ty in range(tiles):
        for tx in range(tiles):
            h = np.bincount(v[ty * T:(ty + 1) * T, tx * T:(tx + 1) * T].ravel(), minlength=256).astype(np.int64)
            clipped = int(np.maximum(h - limit, 0).sum())
            h = np.minimum(h, limit)
            batch = clipped // 256
            residual = clipped - batch * 256
            h += batch
            if residual:
                step = max(256 // residual, 1)
                i = 0
                while i < 256 and residual > 0:
                    h[i] += 1
                    i += step
                    residual -= 1
            lut[ty, tx] = np.clip(np.rint(np.cumsum(h).astype(np.float32) * np.float32(255.0 / area)), 0, 255)
    inv = 1.0 / T
    xs = np.arange(S) * inv - 0.5
    t1 = np.floor(xs).astype(int)
    a = xs - t1
    t2 = np.minimum(t1 + 1, tiles - 1)
    t1 = np.maximum(t1, 0)
    X1, X2, XA = t1[None, :], t2[None, :], a[None, :]
    Y1, Y2, YA = t1[:, None], t2[:, None], a[:, None]
    res = (lut[Y1, X1, v] * (1 - XA) + lut[Y1, X2, v] * XA) * (1 - YA) + (lut[Y2, X1, v] * (1 - XA) + lut[Y2, X2, v] * XA) * YA
    l8 = np.clip(np.rint(res), 0, 255)
    return lab2rgb(l8 * (100.0 / 255.0), A, B)


# ------------------------------------------------------------------ group 2: noise
def iso_noise(x, intensity, color_shift, seed):
    """fpixel.iso_noise: HLS; hue += N(0, color_shift*360*intensity); L += Poisson(std_L*intensity*255)/255*(1-L)."""
    S = x.shape[1]
    h, l, s = rgb2hls(x)
    sd = float(np.std(l.astype(np.float64)))
    pix = np.arange(S * S, dtype=np.uint64).reshape(S, S)
    h = h + color_shift * 360.0 * intensity * gauss(seed ^ 0x5BD1E995, pix, 0)
    h = np.where(h < 0, h + 360.0, h)
    h = np.where(h > 360.0, h - 360.0, h)
    k = poisson_inv(np.float32(sd) * np.float32(intensity) * np.float32(255.0), uni(seed, pix, 7))
    l = l + (k / 255.0) * (1.0 - l)
    return np.clip(hls2rgb(h, l, s), 0, 1)


def gauss_mult_noise(x, gauss_std, mult, seed):
    S = x.shape[1]
    pix = np.arange(S * S, dtype=np.uint64).reshape(S, S)
    out = x * np.asarray(mult).reshape(3, 1, 1)
    if gauss_std > 0:
        out = out + gauss_std * np.stack([gauss(seed, pix, c) for c in range(3)])
    return np.clip(out, 0, 1)


# ------------------------------------------------------------------ group 3: ImageCompression (JPEG)
_QBASE = np.array([
    [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
     14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99],
    [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
     47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32])


def jpeg_tables(quality):
    """IJG jpeg_set_quality: scale 5000/q (q < 50) or 200 - 2q; (base*scale + 50) / 100 clamped to [1, 255]."""
    q = max(int(quality), 1)
    scale = 5000 // q if q < 50 else 200 - 2 * q
    return np.clip((_QBASE * scale + 50) // 100, 1, 255).reshape(2, 8, 8).astype(np.float64)


def _dct_mat():
    u = np.arange(8)[:, None]; k = np.arange(8)[None, :]
    return np.where(u == 0, np.sqrt(0.5), 1.0) * 0.5 * np.cos((2 * k + 1) * u * np.pi / 16)


def jpeg(x, quality):
    """image_compression(".jpg", quality) = cv2.imencode + imdecode, restated: 8-bit RGB -> JFIF YCbCr
    (rounded), 4:2:0 chroma by 2x2 averaging ((sum + 2) >> 2), edge-replicated 16x16 MCUs, 8x8 DCT-II,
    quantise (round to nearest) / dequantise, IDCT, 8-bit samples, h2v2 triangle ("fancy") chroma
    upsampling ((9 a + 3 b + 3 c + d + 8) >> 4), YCbCr -> RGB rounded to 8 bits."""
    S = x.shape[1]
    Sp = 16 * ((S + 15) // 16)
    u8 = np.rint(np.clip(x, 0, 1) * 255.0)
    idx = np.minimum(np.arange(Sp), S - 1)
    P = u8[:, idx][:, :, idx]                                # edge-replicated [3][Sp][Sp]
    r, g, b = P
    Y = np.rint(0.299 * r + 0.587 * g + 0.114 * b)
    Cb = np.clip(np.rint(-0.168736 * r - 0.331264 * g + 0.5 * b + 128), 0, 255)
    Cr = np.clip(np.rint(0.5 * r - 0.418688 * g - 0.081312 * b + 128), 0, 255)
    sub = lambda C: (C.reshape(Sp // 2, 2, Sp // 2, 2).sum((1, 3)).astype(np.int64) + 2) >> 2
    D = _dct_mat()
    Q = jpeg_tables(quality)

    def code(plane, q):
        n = plane.shape[0] // 8
        blk = (plane - 128.0).reshape(n, 8, n, 8).transpose(0, 2, 1, 3)          # [by][bx][y][x]
        F = D @ blk @ D.T
        F = np.rint(F / q) * q
        g_ = D.T @ F @ D
        return np.clip(np.rint(g_ + 128.0), 0, 255).transpose(0, 2, 1, 3).reshape(plane.shape)
    Yr = code(Y, Q[0])
    Cbr, Crr = code(sub(Cb).astype(np.float64), Q[1]), code(sub(Cr).astype(np.float64), Q[1])
    Wc = (S + 1) // 2
    xs = np.arange(S)
    n = xs >> 1
    f = np.clip(np.where(xs & 1, n + 1, n - 1), 0, Wc - 1)

    def up(C):
        C = C.astype(np.int64)
        s = 9 * C[n][:, n] + 3 * C[n][:, f] + 3 * C[f][:, n] + C[f][:, f]
        return ((s + 8) >> 4) - 128.0
    cb, cr = up(Cbr), up(Crr)
    Yv = Yr[:S, :S]
    rgb = np.stack([Yv + 1.402 * cr, Yv - 0.344136 * cb - 0.714136 * cr, Yv + 1.772 * cb])
    return np.clip(np.rint(rgb), 0, 255) / 255.0


# ------------------------------------------------------------------ groups 3-8: the filter pass
def _in_poly5(v, px, py):
    inside = np.zeros(px.shape, bool)
    for i in range(5):
        j = (i + 4) % 5
        xi, yi, xj, yj = v[2 * i], v[2 * i + 1], v[2 * j], v[2 * j + 1]
        with np.errstate(divide="ignore", invalid="ignore"):
            hit = ((yi > py) != (yj > py)) & (px < (xj - xi) * (py - yi) / (yj - yi) + xi)
        inside ^= hit
    return inside


def lit(x, down=1.0, rbc=(1.0, 0.0), shadows=(), shadow_dim=0.5):
    """Downscale (nearest down / nearest up, scale down) then RandomBrightnessContrast (img*alpha + beta,
    clipped) | RandomShadow (pentagons filled even-odd, * (1 - intensity) per polygon)."""
    S = x.shape[1]
    q = np.arange(S)
    if down < 1.0:                                          # float32 expressions of the kernel, same order
        Sd = max(1, int(np.float32(S) * np.float32(down)))
        d = np.minimum(((q.astype(np.float32) * np.float32(Sd)) / np.float32(S)).astype(int), Sd - 1)
        q = np.minimum((((d + np.float32(0.5)).astype(np.float32) * np.float32(S)) / np.float32(Sd)).astype(int), S - 1)
    v = x[:, q][:, :, q]
    v = np.clip(v * rbc[0] + rbc[1], 0, 1)
    py, px = np.mgrid[0:S, 0:S] + 0.5
    for poly in shadows:
        v = np.where(_in_poly5(poly, px, py)[None], np.clip(v * shadow_dim, 0, 1), v)
    return v


def zoom_blur(v, zooms):
    """fblur.zoom_blur: (img + sum_z centre-crop(cv2.resize(img, (int(W z), int(H z)), INTER_LINEAR))) / (n+1)."""
    S = v.shape[1]
    acc = v.copy()
    for z in zooms:
        zs = int(S * np.float32(z))
        off = (zs - S) // 2
        f = (np.arange(S) + off + 0.5) * np.float32(S / zs) - 0.5
        i0 = np.floor(f).astype(int)
        a = f - i0
        a = np.where(i0 < 0, 0.0, a); i0 = np.maximum(i0, 0)
        a = np.where(i0 >= S - 1, 0.0, a); i0 = np.minimum(i0, S - 1)
        i1 = np.minimum(i0 + 1, S - 1)
        rows = v[:, i0] * (1 - a)[None, :, None] + v[:, i1] * a[None, :, None]
        acc = acc + rows[:, :, i0] * (1 - a)[None, None, :] + rows[:, :, i1] * a[None, None, :]
    return acc / (len(zooms) + 1)


def filter2d(v, ker):
    """cv2.filter2D (correlation) with BORDER_REFLECT_101, then clip."""
    S = v.shape[1]
    k = ker.shape[0]
    r = k // 2
    out = np.zeros_like(v)
    for dy in range(-r, r + 1):
        ys = reflect101(np.arange(S) + dy, S)
        for dx in range(-r, r + 1):
            xs = reflect101(np.arange(S) + dx, S)
            out += ker[dy + r, dx + r] * v[:, ys][:, :, xs]
    return np.clip(out, 0, 1)


def snow_bleach(x, snow_point, coeff=2.5):
    """add_snow_bleach: HLS L below snow_point*255/2 + 255/3 (8-bit units) multiplied by brightness_coeff."""
    h, l, s = rgb2hls(x)
    thr = snow_point * 0.5 + 1.0 / 3.0
    low = l < thr
    l2 = np.where(low, np.minimum(l * coeff, 1.0), l)
    return np.where(low[None], hls2rgb(h, l2, s), x)


def rain(x, drops, slant, length=20, color=200 / 255, blur=7, bright=0.7):
    """add_rain ("default"): cv2.line per drop (round-half-up DDA, max(|slant|, length) + 1 points),
    cv2.blur(blur x blur, BORDER_REFLECT_101), HSV V * brightness_coefficient."""
    S = x.shape[1]
    y = x.copy()
    n = max(abs(slant), length)
    for x0, y0 in drops:
        for i in range(n + 1):
            px = x0 + (2 * i * slant + n) // (2 * n)
            py = y0 + (2 * i * length + n) // (2 * n)
            if 0 <= px < S and 0 <= py < S:
                y[:, py, px] = color
    out = filter2d(y, np.full((blur, blur), 1.0 / (blur * blur)))
    return np.clip(out * bright, 0, 1)


# ------------------------------------------------------------------ distortion group (remap of the geometric result)
def remap_bilinear(img, mx, my):
    """cv2.remap(INTER_LINEAR, BORDER_CONSTANT 0) of img [C][S][S] at index coordinates (mx, my)."""
    S = img.shape[1]
    x0, y0 = np.floor(mx).astype(int), np.floor(my).astype(int)
    fx, fy = mx - x0, my - y0
    out = np.zeros((img.shape[0],) + mx.shape)
    for dy in (0, 1):
        for dx in (0, 1):
            xi, yi = x0 + dx, y0 + dy
            w = (fx if dx else 1 - fx) * (fy if dy else 1 - fy)
            ok = (xi >= 0) & (yi >= 0) & (xi < S) & (yi < S)
            out += np.where(ok, w * img[:, np.clip(yi, 0, S - 1), np.clip(xi, 0, S - 1)], 0.0)
    return out


def elastic_field(S, seed, ksize=17, sigma=25.0, alpha=1.0):
    """generate_displacement_fields: standard-normal field per axis (counter RNG, channels 8 / 9), separable
    cv2.GaussianBlur(ksize, sigma, BORDER_REFLECT_101), * alpha -> (dx, dy)."""
    x = np.arange(ksize) - (ksize - 1) / 2
    w = np.exp(-x ** 2 / (2 * sigma ** 2)); w /= w.sum()
    pix = np.arange(S * S, dtype=np.uint64).reshape(S, S)
    out = []
    for c in range(2):
        n = gauss(seed, pix, 8 + c)
        h = sum(w[j] * n[:, reflect101(np.arange(S) + j - ksize // 2, S)] for j in range(ksize))
        v = sum(w[j] * h[reflect101(np.arange(S) + j - ksize // 2, S)] for j in range(ksize))
        out.append(v * alpha)
    return out

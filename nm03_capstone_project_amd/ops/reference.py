"""Plain-PyTorch fp32 references of each pipeline op (the numerics oracle for the HIP kernels,
independent of the C++ golden model). All functions take/return torch tensors on any device."""
import math

import torch
import torch.nn.functional as F


def norm_clip(x, low=0.5, high=2.5, vmin=0.0, vmax=10000.0, cmin=0.68, cmax=4000.0):
    t = (x.float() - vmin) / (vmax - vmin)
    t = t * (high - low) + low
    return t.clamp(cmin, cmax)


def median(img, k=7):
    """Exact k×k median with replicate (clamp-to-edge) padding; img [H, W] float."""
    r = k // 2
    x = F.pad(img[None, None].float(), (r, r, r, r), mode="replicate")
    patches = F.unfold(x, k)  # [1, k*k, H*W]
    return patches.median(dim=1).values.reshape(img.shape)


def gaussian_kernel2d(sigma=0.5, mask=9, dtype=torch.float64):
    r = mask // 2
    ax = torch.arange(-r, r + 1, dtype=dtype)
    g = torch.exp(-(ax[:, None] ** 2 + ax[None, :] ** 2) / (2 * sigma * sigma))
    return g / g.sum()


def sharpen(img, gain=2.0, sigma=0.5, mask=9):
    """Unsharp mask s = c + gain (c − G∗c) in float64 with replicate padding (FAST's 2D form)."""
    r = mask // 2
    x = img.double()[None, None]
    k = gaussian_kernel2d(sigma, mask).to(x.device)[None, None]
    b = F.conv2d(F.pad(x, (r, r, r, r), mode="replicate"), k)[0, 0]
    c = img.double()
    return c + gain * (c - b)


def band(s, lo=0.74, hi=0.91):
    return (s >= lo) & (s <= hi)


def threshold(x, lo, hi):
    """BinaryThresholding reference: lo ≤ x ≤ hi → 1 (uint8)."""
    return ((x >= lo) & (x <= hi)).to(torch.uint8)


def dilate(mask, size=3):
    r = size // 2
    x = mask.float()[None, None]
    return (F.max_pool2d(x, size, stride=1, padding=r)[0, 0] > 0.5)


def erode(mask, size=3):
    # max_pool2d pads with -inf, i.e. out-of-image samples never win: "ignored" (App. A.7).
    r = size // 2
    x = (1.0 - mask.float())[None, None]
    return ~(F.max_pool2d(x, size, stride=1, padding=r)[0, 0] > 0.5)


def disc_se(size, dims=2):
    """The digital disc (dims=2) / ball (dims=3) of radius size // 2: offsets with |d|² ≤ r²."""
    r = size // 2
    ax = torch.arange(-r, r + 1, dtype=torch.int64)
    grids = torch.meshgrid(*([ax] * dims), indexing="ij")
    return sum(g * g for g in grids) <= r * r


def dilate_disc(mask, size=3):
    """Binary dilation with the disc SE as a conv2d count (zero padding = out-of-image ignored)."""
    r = size // 2
    k = disc_se(size).to(torch.float64)[None, None].to(mask.device)
    return F.conv2d(mask.to(torch.float64)[None, None], k, padding=r)[0, 0] > 0.5


def erode_disc(mask, size=3):
    """Binary erosion with the disc SE: every in-image sample under the disc set. Out-of-image samples
    are ignored: the count of set samples equals the count of in-image samples under the disc."""
    r = size // 2
    k = disc_se(size).to(torch.float64)[None, None].to(mask.device)
    hits = F.conv2d(mask.to(torch.float64)[None, None], k, padding=r)[0, 0]
    inside = F.conv2d(torch.ones_like(mask, dtype=torch.float64)[None, None], k, padding=r)[0, 0]
    return hits > inside - 0.5


def dilate_ball(mask, size=7):
    """3D binary dilation with the ball SE as a conv3d count, [D, H, W]."""
    r = size // 2
    k = disc_se(size, 3).to(torch.float64)[None, None].to(mask.device)
    return F.conv3d(mask.to(torch.float64)[None, None], k, padding=r)[0, 0] > 0.5


def border(mask, radius=2):
    return mask & ~erode(mask, 2 * radius + 1)


def region_grow(bnd, seeds, connectivity=4):
    """Geodesic reconstruction: iterate R ← band ∧ dilate(R) from the in-band seeds to a fixpoint."""
    h, w = bnd.shape
    reg = torch.zeros_like(bnd)
    for (x, y, *_rest) in seeds:
        if 0 <= x < w and 0 <= y < h and bnd[y, x]:
            reg[y, x] = True
    if connectivity == 4:
        k = torch.tensor([[0, 1, 0], [1, 1, 1], [0, 1, 0]], dtype=torch.float32, device=bnd.device)
    else:
        k = torch.ones((3, 3), dtype=torch.float32, device=bnd.device)
    while True:
        grown = F.conv2d(reg.float()[None, None], k[None, None], padding=1)[0, 0] > 0
        nxt = grown & bnd
        if torch.equal(nxt, reg):
            return reg
        reg = nxt


def render_gray(values, lo, hi, out_w=512, out_h=512, nearest=False):
    """Bilinear 2× (generally: fit) render of an [H, W] float image onto out_h×out_w, f32 math
    in the contract order (pixel_math.h), window [lo, hi] → uint8. `nearest`: the source pixel under
    each canvas pixel's centre instead (--render-filter nearest)."""
    h, w = values.shape
    scale = min(out_w / w, out_h / h)
    ox, oy = (out_w - w * scale) / 2, (out_h - h * scale) / 2
    dev = values.device
    u = torch.arange(out_w, device=dev, dtype=torch.float32)
    v = torch.arange(out_h, device=dev, dtype=torch.float32)
    sx = (u + 0.5 - ox) * (1.0 / scale)
    sy = (v + 0.5 - oy) * (1.0 / scale)
    fx, fy = sx - 0.5, sy - 0.5
    x0, y0 = torch.floor(fx), torch.floor(fy)
    wx, wy = fx - x0, fy - y0
    x0i, y0i = x0.long(), y0.long()
    xa, xb = x0i.clamp(0, w - 1), (x0i + 1).clamp(0, w - 1)
    ya, yb = y0i.clamp(0, h - 1), (y0i + 1).clamp(0, h - 1)
    a = values[ya][:, xa]
    b = values[ya][:, xb]
    c = values[yb][:, xa]
    d = values[yb][:, xb]
    top = (1 - wx) * a + wx * b
    bot = (1 - wx) * c + wx * d
    val = (1 - wy)[:, None] * top + wy[:, None] * bot
    if nearest:
        val = values[torch.floor(sy).long().clamp(0, h - 1)][:, torch.floor(sx).long().clamp(0, w - 1)]
    inv = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(hi - lo, dtype=torch.float32) if hi > lo else torch.tensor(0.0)
    g = ((val - lo) * inv.to(val.device)).clamp(0, 1)
    out = torch.floor(g * 255 + 0.5).to(torch.uint8)
    inside = ((sx >= 0) & (sx < w))[None, :] & ((sy >= 0) & (sy < h))[:, None]
    return torch.where(inside, out, torch.zeros_like(out))


def render_labels(label, brd, fill=153, border_value=255, out_w=512, out_h=512):
    h, w = label.shape
    scale = min(out_w / w, out_h / h)
    ox, oy = (out_w - w * scale) / 2, (out_h - h * scale) / 2
    dev = label.device
    sx = (torch.arange(out_w, device=dev, dtype=torch.float32) + 0.5 - ox) / scale
    sy = (torch.arange(out_h, device=dev, dtype=torch.float32) + 0.5 - oy) / scale
    xi = torch.floor(sx).long().clamp(0, w - 1)
    yi = torch.floor(sy).long().clamp(0, h - 1)
    lab = label[yi][:, xi]
    bd = brd[yi][:, xi]
    out = torch.where(bd, torch.full_like(lab, border_value, dtype=torch.uint8),
                      torch.where(lab, torch.full_like(lab, fill, dtype=torch.uint8),
                                  torch.zeros_like(lab, dtype=torch.uint8)))
    inside = ((sx >= 0) & (sx < w))[None, :] & ((sy >= 0) & (sy < h))[:, None]
    return torch.where(inside, out, torch.zeros_like(out))


def psnr(a, b):
    mse = ((a.double() - b.double()) ** 2).mean().item()
    return math.inf if mse == 0 else 10 * math.log10(255.0 ** 2 / mse)

"""``paddle.vision.transforms`` (reference `python/paddle/vision/transforms/transforms.py` and
`functional.py`). Works on HWC numpy images (the reference's 'cv2' backend) and CHW tensors."""
from __future__ import annotations

import math
import numbers
import random

import numpy as np
import torch
import torch.nn.functional as F


def _is_tensor(x):
    return isinstance(x, torch.Tensor)


def _hw(img):
    if _is_tensor(img):
        return img.shape[-2], img.shape[-1]
    return img.shape[0], img.shape[1]


# ------------------------------------------------------------------------------------ functional
def to_tensor(pic, data_format="CHW"):
    if _is_tensor(pic):
        return pic
    arr = np.asarray(pic)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if t.dtype == torch.uint8:
        t = t.float() / 255.0
    else:
        t = t.float()
    return t.permute(2, 0, 1).contiguous() if data_format == "CHW" else t


def resize(img, size, interpolation="bilinear"):
    h, w = _hw(img)
    if isinstance(size, int):
        if h < w:
            oh, ow = size, int(size * w / h)
        else:
            oh, ow = int(size * h / w), size
    else:
        oh, ow = size
    t = img if _is_tensor(img) else torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)
    dt = t.dtype
    mode = {"bilinear": "bilinear", "nearest": "nearest", "bicubic": "bicubic"}.get(interpolation, "bilinear")
    out = F.interpolate(t.unsqueeze(0).float(), (oh, ow), mode=mode,
                        align_corners=False if mode != "nearest" else None)[0]
    if dt == torch.uint8:
        out = out.round().clamp(0, 255).to(torch.uint8)
    return out if _is_tensor(img) else out.permute(1, 2, 0).numpy()


def crop(img, top, left, height, width):
    if _is_tensor(img):
        return img[..., top:top + height, left:left + width]
    return img[top:top + height, left:left + width]


def center_crop(img, output_size):
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    h, w = _hw(img)
    return crop(img, int(round((h - oh) / 2.0)), int(round((w - ow) / 2.0)), oh, ow)


def hflip(img):
    return img.flip(-1) if _is_tensor(img) else img[:, ::-1]


def vflip(img):
    return img.flip(-2) if _is_tensor(img) else img[::-1]


def pad(img, padding, fill=0, padding_mode="constant"):
    if isinstance(padding, int):
        padding = (padding,) * 4
    elif len(padding) == 2:
        padding = (padding[0], padding[1], padding[0], padding[1])
    l, t, r, b = padding
    if _is_tensor(img):
        mode = {"constant": "constant", "edge": "replicate", "reflect": "reflect", "symmetric": "reflect"}[padding_mode]
        x = img.unsqueeze(0).float() if mode != "constant" else img
        out = F.pad(x, (l, r, t, b), mode=mode, value=fill) if mode == "constant" else F.pad(x, (l, r, t, b), mode=mode)[0]
        return out.to(img.dtype)
    pw = ((t, b), (l, r)) + (((0, 0),) if img.ndim == 3 else ())
    if padding_mode == "constant":
        return np.pad(img, pw, mode="constant", constant_values=fill)
    return np.pad(img, pw, mode={"edge": "edge", "reflect": "reflect", "symmetric": "symmetric"}[padding_mode])


def normalize(img, mean, std, data_format="CHW", to_rgb=False):
    if _is_tensor(img):
        m = torch.as_tensor(mean, dtype=img.dtype, device=img.device)
        s = torch.as_tensor(std, dtype=img.dtype, device=img.device)
        if data_format == "CHW":
            return (img - m[:, None, None]) / s[:, None, None]
        return (img - m) / s
    img = np.asarray(img, dtype=np.float32)
    return (img - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)


def adjust_brightness(img, factor):
    return _blend(img, np.zeros_like(img) if not _is_tensor(img) else torch.zeros_like(img), factor)


def _gray(img):
    if _is_tensor(img):
        return (0.299 * img[0] + 0.587 * img[1] + 0.114 * img[2]).expand_as(img)
    g = img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114
    return np.repeat(g[..., None], img.shape[-1], -1)


def _blend(a, b, factor):
    out = a * factor + b * (1 - factor)
    if _is_tensor(a):
        return out.clamp(0, 1 if a.is_floating_point() else 255).to(a.dtype)
    return np.clip(out, 0, 255 if a.dtype == np.uint8 else 1).astype(a.dtype)


def adjust_contrast(img, factor):
    g = _gray(img)
    mean = g.mean() if _is_tensor(img) else np.mean(g)
    return _blend(img, (torch.full_like(img, float(mean)) if _is_tensor(img) else np.full_like(img, mean)), factor)


def adjust_saturation(img, factor):
    return _blend(img, _gray(img), factor)


def adjust_hue(img, hue_factor):
    if hue_factor == 0:
        return img
    t = img.float() if _is_tensor(img) else torch.from_numpy(np.asarray(img, np.float32) / (255.0 if np.asarray(img).dtype == np.uint8 else 1.0)).permute(2, 0, 1)
    r, g, b = t[0], t[1], t[2]
    mx, _ = t.max(0)
    mn, _ = t.min(0)
    d = mx - mn + 1e-12
    h = torch.where(mx == r, ((g - b) / d) % 6, torch.where(mx == g, (b - r) / d + 2, (r - g) / d + 4)) / 6.0
    s = (mx - mn) / (mx + 1e-12)
    v = mx
    h = (h + hue_factor) % 1.0
    i = (h * 6).floor()
    f = h * 6 - i
    p, q, tt = v * (1 - s), v * (1 - f * s), v * (1 - (1 - f) * s)
    i = i.long() % 6
    rr = torch.stack([v, q, p, p, tt, v])
    gg = torch.stack([tt, v, v, q, p, p])
    bb = torch.stack([p, p, tt, v, v, q])
    out = torch.stack([x.gather(0, i.unsqueeze(0))[0] for x in (rr, gg, bb)])
    if _is_tensor(img):
        return out.to(img.dtype)
    arr = out.permute(1, 2, 0).numpy()
    return (arr * 255).round().astype(np.uint8) if np.asarray(img).dtype == np.uint8 else arr


def rotate(img, angle, interpolation="nearest", expand=False, center=None, fill=0):
    t = img if _is_tensor(img) else torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)
    dt = t.dtype
    a = math.radians(-angle)
    theta = torch.tensor([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0]])
    grid = F.affine_grid(theta[None], [1, *t.shape], align_corners=False)
    out = F.grid_sample(t[None].float(), grid, mode="nearest" if interpolation == "nearest" else "bilinear",
                        align_corners=False, padding_mode="zeros")[0].to(dt)
    return out if _is_tensor(img) else out.permute(1, 2, 0).numpy()


def to_grayscale(img, num_output_channels=1):
    g = _gray(img)
    if _is_tensor(img):
        return g[:1] if num_output_channels == 1 else g
    return g[..., :1] if num_output_channels == 1 else g


# ------------------------------------------------------------------------------------ classes
class BaseTransform:
    def __init__(self, keys=None):
        self.keys = keys

    def _apply_image(self, img):
        raise NotImplementedError

    def __call__(self, inputs):
        if isinstance(inputs, tuple):
            return (self._apply_image(inputs[0]),) + tuple(inputs[1:])
        return self._apply_image(inputs)


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data


class ToTensor(BaseTransform):
    def __init__(self, data_format="CHW", keys=None):
        super().__init__(keys)
        self.data_format = data_format

    def _apply_image(self, img):
        return to_tensor(img, self.data_format)


class Resize(BaseTransform):
    def __init__(self, size, interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size, self.interpolation = size, interpolation

    def _apply_image(self, img):
        return resize(img, self.size, self.interpolation)


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        super().__init__(keys)
        self.size = size

    def _apply_image(self, img):
        return center_crop(img, self.size)


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else size
        self.padding, self.pad_if_needed, self.fill, self.padding_mode = padding, pad_if_needed, fill, padding_mode

    def _apply_image(self, img):
        if self.padding is not None:
            img = pad(img, self.padding, self.fill, self.padding_mode)
        h, w = _hw(img)
        th, tw = self.size
        if self.pad_if_needed and (h < th or w < tw):
            img = pad(img, (max(tw - w, 0), max(th - h, 0)), self.fill, self.padding_mode)
            h, w = _hw(img)
        i, j = random.randint(0, h - th), random.randint(0, w - tw)
        return crop(img, i, j, th, tw)


class RandomResizedCrop(BaseTransform):
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3. / 4, 4. / 3), interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else size
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def _apply_image(self, img):
        h, w = _hw(img)
        area = h * w
        for _ in range(10):
            ta = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            cw, ch = int(round(math.sqrt(ta * ar))), int(round(math.sqrt(ta / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                i, j = random.randint(0, h - ch), random.randint(0, w - cw)
                return resize(crop(img, i, j, ch, cw), self.size, self.interpolation)
        return resize(center_crop(img, min(h, w)), self.size, self.interpolation)


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return hflip(img) if random.random() < self.prob else img


class RandomVerticalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return vflip(img) if random.random() < self.prob else img


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format="CHW", to_rgb=False, keys=None):
        super().__init__(keys)
        self.mean = [mean] * 3 if isinstance(mean, numbers.Number) else mean
        self.std = [std] * 3 if isinstance(std, numbers.Number) else std
        self.data_format, self.to_rgb = data_format, to_rgb

    def _apply_image(self, img):
        return normalize(img, self.mean, self.std, self.data_format, self.to_rgb)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        super().__init__(keys)
        self.order = order

    def _apply_image(self, img):
        if _is_tensor(img):
            return img.permute(*self.order)
        if img.ndim == 2:
            img = img[..., None]
        return img.transpose(self.order)


class Pad(BaseTransform):
    def __init__(self, padding, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.padding, self.fill, self.padding_mode = padding, fill, padding_mode

    def _apply_image(self, img):
        return pad(img, self.padding, self.fill, self.padding_mode)


class BrightnessTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_brightness(img, random.uniform(max(0, 1 - self.value), 1 + self.value)) if self.value else img


class ContrastTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_contrast(img, random.uniform(max(0, 1 - self.value), 1 + self.value)) if self.value else img


class SaturationTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_saturation(img, random.uniform(max(0, 1 - self.value), 1 + self.value)) if self.value else img


class HueTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        return adjust_hue(img, random.uniform(-self.value, self.value)) if self.value else img


class ColorJitter(BaseTransform):
    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0, keys=None):
        super().__init__(keys)
        self.ts = [BrightnessTransform(brightness), ContrastTransform(contrast),
                   SaturationTransform(saturation), HueTransform(hue)]

    def _apply_image(self, img):
        for t in random.sample(self.ts, len(self.ts)):
            img = t._apply_image(img)
        return img


class RandomRotation(BaseTransform):
    def __init__(self, degrees, interpolation="nearest", expand=False, center=None, fill=0, keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.interpolation = interpolation

    def _apply_image(self, img):
        return rotate(img, random.uniform(*self.degrees), self.interpolation)


class Grayscale(BaseTransform):
    def __init__(self, num_output_channels=1, keys=None):
        super().__init__(keys)
        self.n = num_output_channels

    def _apply_image(self, img):
        return to_grayscale(img, self.n)


class RandomErasing(BaseTransform):
    def __init__(self, prob=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3), value=0, inplace=False, keys=None):
        super().__init__(keys)
        self.prob, self.scale, self.ratio, self.value = prob, scale, ratio, value

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        h, w = _hw(img)
        for _ in range(10):
            ea = h * w * random.uniform(*self.scale)
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            eh, ew = int(round(math.sqrt(ea * ar))), int(round(math.sqrt(ea / ar)))
            if eh < h and ew < w:
                i, j = random.randint(0, h - eh), random.randint(0, w - ew)
                img = img.clone() if _is_tensor(img) else img.copy()
                if _is_tensor(img):
                    img[..., i:i + eh, j:j + ew] = self.value
                else:
                    img[i:i + eh, j:j + ew] = self.value
                return img
        return img


# ------------------------------------------------------------------------------------ affine / perspective
def _warp(img, inv_map, interpolation, fill):
    """Sample ``img`` at inverse-mapped pixel centres: inv_map(x, y) -> (src_x, src_y) arrays."""
    t = img if _is_tensor(img) else torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)
    dt = t.dtype
    C, H, W = t.shape
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float64) + 0.5,
                            torch.arange(W, dtype=torch.float64) + 0.5, indexing="ij")
    sx, sy = inv_map(xs, ys)
    grid = torch.stack([sx / W * 2 - 1, sy / H * 2 - 1], -1).float()[None]
    src = t[None].float()
    mode = "nearest" if interpolation == "nearest" else "bilinear"
    out = F.grid_sample(src, grid, mode=mode, padding_mode="zeros", align_corners=False)[0]
    if fill:
        ones = torch.ones(1, 1, H, W)
        cover = F.grid_sample(ones, grid, mode=mode, padding_mode="zeros", align_corners=False)[0]
        out = out + (1 - cover) * torch.as_tensor(fill, dtype=torch.float32).reshape(-1, 1, 1)
    out = out.round().clamp(0, 255).to(dt) if not dt.is_floating_point else out.to(dt)
    return out if _is_tensor(img) else out.permute(1, 2, 0).numpy()


def _affine_matrix(center, angle, translate, scale, shear):
    """Forward 2x3 matrix (reference functional._get_affine_matrix): T(center+translate) · R·Sh·S ·
    T(−center), angle / shear in degrees (clockwise image rotation like the reference)."""
    cx, cy = center
    tx, ty = translate
    rot = math.radians(angle)
    sx, sy = (math.radians(shear[0]), math.radians(shear[1])) if isinstance(shear, (list, tuple)) \
        else (math.radians(shear), 0.0)
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = np.array([[a, b, 0.0], [c, d, 0.0]]) * scale
    m[0, 2] = cx + tx - (m[0, 0] * cx + m[0, 1] * cy)
    m[1, 2] = cy + ty - (m[1, 0] * cx + m[1, 1] * cy)
    return m


def affine(img, angle, translate, scale, shear, interpolation="nearest", fill=0, center=None):
    """Reference `vision/transforms/functional.py:affine`."""
    H, W = _hw(img)
    center = center if center is not None else (W * 0.5, H * 0.5)
    m = np.vstack([_affine_matrix(center, angle, translate, scale, shear), [0, 0, 1]])
    inv = np.linalg.inv(m)

    def inv_map(x, y):
        return inv[0, 0] * x + inv[0, 1] * y + inv[0, 2], inv[1, 0] * x + inv[1, 1] * y + inv[1, 2]
    return _warp(img, inv_map, interpolation, fill)


def _homography(src, dst):
    """3x3 H with H·src_i ∝ dst_i for 4 point pairs."""
    A, b = [], []
    for (x, y), (u, v) in zip(src, dst):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y])
        b += [u, v]
    h = np.linalg.solve(np.asarray(A, dtype=np.float64), np.asarray(b, dtype=np.float64))
    return np.append(h, 1.0).reshape(3, 3)


def perspective(img, startpoints, endpoints, interpolation="nearest", fill=0):
    """Reference `vision/transforms/functional.py:perspective`: the image plane warped so
    ``startpoints`` (4 corners, [x, y]) land on ``endpoints``."""
    Hm = _homography(endpoints, startpoints)  # output pixel -> source pixel

    def inv_map(x, y):
        w = Hm[2, 0] * x + Hm[2, 1] * y + Hm[2, 2]
        return (Hm[0, 0] * x + Hm[0, 1] * y + Hm[0, 2]) / w, (Hm[1, 0] * x + Hm[1, 1] * y + Hm[1, 2]) / w
    return _warp(img, inv_map, interpolation, fill)


def erase(img, i, j, h, w, v, inplace=False):
    """Reference `vision/transforms/functional.py:erase`: region [i:i+h, j:j+w] set to ``v``."""
    out = img if inplace else (img.clone() if _is_tensor(img) else img.copy())
    if _is_tensor(out):
        out[..., i:i + h, j:j + w] = torch.as_tensor(v, dtype=out.dtype) if not isinstance(v, numbers.Number) else v
    else:
        out[i:i + h, j:j + w] = v
    return out


class RandomAffine(BaseTransform):
    """Reference `transforms.py:RandomAffine`."""

    def __init__(self, degrees, translate=None, scale=None, shear=None, interpolation="nearest",
                 fill=0, center=None, keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else tuple(degrees)
        self.translate, self.scale, self.interpolation, self.fill, self.center = \
            translate, scale, interpolation, fill, center
        if shear is not None and isinstance(shear, numbers.Number):
            shear = (-shear, shear)
        self.shear = shear

    def _params(self, h, w):
        angle = random.uniform(*self.degrees)
        tx = ty = 0.0
        if self.translate is not None:
            tx = round(random.uniform(-self.translate[0] * w, self.translate[0] * w))
            ty = round(random.uniform(-self.translate[1] * h, self.translate[1] * h))
        sc = random.uniform(*self.scale) if self.scale is not None else 1.0
        sh = (0.0, 0.0)
        if self.shear is not None:
            sh = (random.uniform(self.shear[0], self.shear[1]),
                  random.uniform(self.shear[2], self.shear[3]) if len(self.shear) == 4 else 0.0)
        return angle, (tx, ty), sc, sh

    def _apply_image(self, img):
        h, w = _hw(img)
        angle, tr, sc, sh = self._params(h, w)
        return affine(img, angle, tr, sc, sh, self.interpolation, self.fill, self.center)


class RandomPerspective(BaseTransform):
    """Reference `transforms.py:RandomPerspective`."""

    def __init__(self, prob=0.5, distortion_scale=0.5, interpolation="nearest", fill=0, keys=None):
        super().__init__(keys)
        self.prob, self.d, self.interpolation, self.fill = prob, distortion_scale, interpolation, fill

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        h, w = _hw(img)
        dh, dw = int(self.d * h / 2), int(self.d * w / 2)
        tl = (random.randint(0, dw), random.randint(0, dh))
        tr = (w - 1 - random.randint(0, dw), random.randint(0, dh))
        br = (w - 1 - random.randint(0, dw), h - 1 - random.randint(0, dh))
        bl = (random.randint(0, dw), h - 1 - random.randint(0, dh))
        start = [(0, 0), (w - 1, 0), (w - 1, h - 1), (0, h - 1)]
        return perspective(img, start, [tl, tr, br, bl], self.interpolation, self.fill)

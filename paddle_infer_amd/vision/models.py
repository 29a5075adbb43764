"""``paddle.vision.models`` (reference `python/paddle/vision/models/*.py`): LeNet, AlexNet, VGG,
ResNet / ResNeXt / wide ResNet, MobileNetV1/V2/V3, SqueezeNet, ShuffleNetV2, DenseNet, GoogLeNet.
Built from this framework's layers (convolutions/BN run on MIOpen through torch; bf16 AMP and
``channels_last`` tensors are the MI355X-friendly setting). ``pretrained=True`` is not
available offline and raises."""
from __future__ import annotations

import torch

from .. import nn


def _no_pretrained(pretrained):
    if pretrained:
        raise RuntimeError("pretrained weights need a download; not available offline")


def _cbr(cin, cout, k, s=1, p=0, groups=1, act="relu"):
    layers = [nn.Conv2D(cin, cout, k, s, p, groups=groups, bias_attr=False), nn.BatchNorm2D(cout)]
    if act == "relu":
        layers.append(nn.ReLU())
    elif act == "relu6":
        layers.append(nn.ReLU6())
    elif act == "hardswish":
        layers.append(nn.Hardswish())
    elif act == "swish":
        layers.append(nn.Swish())
    return nn.Sequential(*layers)


# ----------------------------------------------------------------------------------------- LeNet
class LeNet(nn.Layer):
    def __init__(self, num_classes=10):
        super().__init__()
        self.num_classes = num_classes
        self.features = nn.Sequential(nn.Conv2D(1, 6, 3, 1, 1), nn.ReLU(), nn.MaxPool2D(2, 2),
                                      nn.Conv2D(6, 16, 5, 1, 0), nn.ReLU(), nn.MaxPool2D(2, 2))
        if num_classes > 0:
            self.fc = nn.Sequential(nn.Linear(400, 120), nn.Linear(120, 84), nn.Linear(84, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.num_classes > 0:
            x = self.fc(torch.flatten(x, 1))
        return x


# ----------------------------------------------------------------------------------------- AlexNet
class AlexNet(nn.Layer):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.num_classes = num_classes
        self.features = nn.Sequential(
            nn.Conv2D(3, 64, 11, 4, 2), nn.ReLU(), nn.MaxPool2D(3, 2),
            nn.Conv2D(64, 192, 5, padding=2), nn.ReLU(), nn.MaxPool2D(3, 2),
            nn.Conv2D(192, 384, 3, padding=1), nn.ReLU(), nn.Conv2D(384, 256, 3, padding=1), nn.ReLU(),
            nn.Conv2D(256, 256, 3, padding=1), nn.ReLU(), nn.MaxPool2D(3, 2))
        self.avgpool = nn.AdaptiveAvgPool2D((6, 6))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(256 * 36, 4096), nn.ReLU(),
                                            nn.Dropout(), nn.Linear(4096, 4096), nn.ReLU(),
                                            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(torch.flatten(x, 1)) if self.num_classes > 0 else x


def alexnet(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return AlexNet(**kw)


# ----------------------------------------------------------------------------------------- VGG
_VGG = {11: [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        13: [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
        19: [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]}


def make_vgg_features(cfg, batch_norm=False):
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2D(2, 2))
        else:
            layers.append(nn.Conv2D(cin, v, 3, padding=1))
            if batch_norm:
                layers.append(nn.BatchNorm2D(v))
            layers.append(nn.ReLU())
            cin = v
    return nn.Sequential(*layers)


class VGG(nn.Layer):
    def __init__(self, features, num_classes=1000, with_pool=True):
        super().__init__()
        self.features, self.num_classes, self.with_pool = features, num_classes, with_pool
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((7, 7))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(512 * 49, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        return self.classifier(torch.flatten(x, 1)) if self.num_classes > 0 else x


def _vgg(depth, batch_norm, pretrained, **kw):
    _no_pretrained(pretrained)
    return VGG(make_vgg_features(_VGG[depth], batch_norm), **kw)


def vgg11(pretrained=False, batch_norm=False, **kw): return _vgg(11, batch_norm, pretrained, **kw)
def vgg13(pretrained=False, batch_norm=False, **kw): return _vgg(13, batch_norm, pretrained, **kw)
def vgg16(pretrained=False, batch_norm=False, **kw): return _vgg(16, batch_norm, pretrained, **kw)
def vgg19(pretrained=False, batch_norm=False, **kw): return _vgg(19, batch_norm, pretrained, **kw)


# ----------------------------------------------------------------------------------------- ResNet
def _residual_join(x, downsample=None):
    """A residual-gradient join (ops/conv.py ResidualGradJoin): the first conv's data-gradient
    epilogue adds the other consumer's gradient of the block input — the residual BatchNorm's
    (identity shortcut) or the shortcut conv's (downsampling block, ``_downsample_join``) — so
    autograd does not sum the two with a separate add. None where it does not apply (CPU, no
    autograd)."""
    from ..ops import conv as _conv
    if downsample is not None or not (_conv.RES_JOIN and x.is_cuda and torch.is_grad_enabled()):
        return None
    return _conv.ResidualGradJoin()


# PIAMD_DS_JOIN=0: downsampling blocks sum their two block-input gradients with an autograd add
DS_JOIN = __import__("os").environ.get("PIAMD_DS_JOIN", "1") != "0"


def _downsample_join(x, downsample):
    """Join for a downsampling block: the shortcut conv (run after the main path, so its
    backward comes first) gives its input gradient to the main path's first conv."""
    if downsample is None or not DS_JOIN:
        return None
    return _residual_join(x)


class _Give:
    """``with _Give(j)``: the next conv gives its input gradient to the join ``j`` (no-op for
    None)."""

    def __init__(self, j):
        self.cm = None
        if j is not None:
            from ..ops import conv as _conv
            self.cm = _conv.join_give(j)

    def __enter__(self):
        if self.cm is not None:
            self.cm.__enter__()

    def __exit__(self, *exc):
        if self.cm is not None:
            self.cm.__exit__(*exc)
        return False


class _Joined:
    """``with _Joined(j, source=True)``: the next conv (source) / residual BatchNorm (sink) uses
    the join ``j`` (no-op for None)."""

    def __init__(self, j, source):
        self.cm = None
        if j is not None:
            from ..ops import batchnorm as _bn, conv as _conv
            self.cm = _conv.join_source(j) if source else _bn.join_sink(j)

    def __enter__(self):
        if self.cm is not None:
            self.cm.__enter__()

    def __exit__(self, *exc):
        if self.cm is not None:
            self.cm.__exit__(*exc)
        return False


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super().__init__()
        self.conv1 = nn.Conv2D(inplanes, planes, 3, stride, 1, bias_attr=False)
        self.bn1 = nn.BatchNorm2D(planes)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, 1, 1, bias_attr=False)
        self.bn2 = nn.BatchNorm2D(planes)
        self.downsample = downsample

    def forward(self, x):
        j = _residual_join(x, self.downsample)
        jd = _downsample_join(x, self.downsample)
        with _Joined(j or jd, source=True):
            h = self.conv1(x)
        out = self.bn1(h, act="relu")                              # fused BN + ReLU
        h = self.conv2(out)
        with _Give(jd):  # the shortcut after the main path: its backward runs first
            idt = x if self.downsample is None else self.downsample(x)
        with _Joined(j, source=False):
            return self.bn2(h, residual=idt, act="relu")           # fused BN + add + ReLU


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False)
        self.bn1 = nn.BatchNorm2D(width)
        self.conv2 = nn.Conv2D(width, width, 3, stride, dilation, dilation=dilation, groups=groups,
                               bias_attr=False)
        self.bn2 = nn.BatchNorm2D(width)
        self.conv3 = nn.Conv2D(width, planes * 4, 1, bias_attr=False)
        self.bn3 = nn.BatchNorm2D(planes * 4)
        self.relu = nn.ReLU()
        self.downsample = downsample

    def forward(self, x):
        j = _residual_join(x, self.downsample)
        jd = _downsample_join(x, self.downsample)
        with _Joined(j or jd, source=True):
            h = self.conv1(x)
        out = self.bn1(h, act="relu")
        out = self.bn2(self.conv2(out), act="relu")
        h = self.conv3(out)
        with _Give(jd):  # the shortcut after the main path: its backward runs first
            idt = x if self.downsample is None else self.downsample(x)
        with _Joined(j, source=False):
            return self.bn3(h, residual=idt, act="relu")  # fused BN + add + ReLU


class ResNet(nn.Layer):
    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1):
        super().__init__()
        cfg = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3],
               152: [3, 8, 36, 3]}[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self.inplanes = 64
        self.conv1 = nn.Conv2D(3, 64, 7, 2, 3, bias_attr=False)
        self.bn1 = nn.BatchNorm2D(64)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, cfg[0])
        self.layer2 = self._make_layer(block, 128, cfg[1], 2)
        self.layer3 = self._make_layer(block, 256, cfg[2], 2)
        self.layer4 = self._make_layer(block, 512, cfg[3], 2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1))
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride, bias_attr=False),
                                 nn.BatchNorm2D(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.bn1(self.conv1(x), act="relu"))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.fc(torch.flatten(x, 1))
        return x


def _resnet(block, depth, pretrained, **kw):
    _no_pretrained(pretrained)
    return ResNet(block, depth, **kw)


def resnet18(pretrained=False, **kw): return _resnet(BasicBlock, 18, pretrained, **kw)
def resnet34(pretrained=False, **kw): return _resnet(BasicBlock, 34, pretrained, **kw)
def resnet50(pretrained=False, **kw): return _resnet(BottleneckBlock, 50, pretrained, **kw)
def resnet101(pretrained=False, **kw): return _resnet(BottleneckBlock, 101, pretrained, **kw)
def resnet152(pretrained=False, **kw): return _resnet(BottleneckBlock, 152, pretrained, **kw)
def resnext50_32x4d(pretrained=False, **kw): return _resnet(BottleneckBlock, 50, pretrained, width=4, groups=32, **kw)
def resnext50_64x4d(pretrained=False, **kw): return _resnet(BottleneckBlock, 50, pretrained, width=4, groups=64, **kw)
def resnext101_32x4d(pretrained=False, **kw): return _resnet(BottleneckBlock, 101, pretrained, width=4, groups=32, **kw)
def resnext101_64x4d(pretrained=False, **kw): return _resnet(BottleneckBlock, 101, pretrained, width=4, groups=64, **kw)
def resnext152_32x4d(pretrained=False, **kw): return _resnet(BottleneckBlock, 152, pretrained, width=4, groups=32, **kw)
def resnext152_64x4d(pretrained=False, **kw): return _resnet(BottleneckBlock, 152, pretrained, width=4, groups=64, **kw)
def wide_resnet50_2(pretrained=False, **kw): return _resnet(BottleneckBlock, 50, pretrained, width=128, **kw)
def wide_resnet101_2(pretrained=False, **kw): return _resnet(BottleneckBlock, 101, pretrained, width=128, **kw)


# ----------------------------------------------------------------------------------------- MobileNet
class MobileNetV1(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        c = lambda v: int(v * scale)  # noqa: E731
        cfg = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2)] + \
              [(512, 512, 1)] * 5 + [(512, 1024, 2), (1024, 1024, 1)]
        layers = [_cbr(3, c(32), 3, 2, 1)]
        for cin, cout, s in cfg:
            layers += [_cbr(c(cin), c(cin), 3, s, 1, groups=c(cin)), _cbr(c(cin), c(cout), 1)]
        self.features = nn.Sequential(*layers)
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(c(1024), num_classes)

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool(x)
        return self.fc(torch.flatten(x, 1)) if self.num_classes > 0 else x


class _InvertedResidual(nn.Layer):
    def __init__(self, cin, cout, stride, expand):
        super().__init__()
        hidden = int(round(cin * expand))
        self.use_res = stride == 1 and cin == cout
        layers = [] if expand == 1 else [_cbr(cin, hidden, 1, act="relu6")]
        layers += [_cbr(hidden, hidden, 3, stride, 1, groups=hidden, act="relu6"),
                   nn.Conv2D(hidden, cout, 1, bias_attr=False), nn.BatchNorm2D(cout)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


def _div8(v):
    return max(8, int(v + 4) // 8 * 8)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1),
               (6, 160, 3, 2), (6, 320, 1, 1)]
        cin = _div8(32 * scale)
        last = _div8(1280 * max(1.0, scale))
        layers = [_cbr(3, cin, 3, 2, 1, act="relu6")]
        for t, c, n, s in cfg:
            cout = _div8(c * scale)
            for i in range(n):
                layers.append(_InvertedResidual(cin, cout, s if i == 0 else 1, t))
                cin = cout
        layers.append(_cbr(cin, last, 1, act="relu6"))
        self.features = nn.Sequential(*layers)
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(last, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        return self.classifier(torch.flatten(x, 1)) if self.num_classes > 0 else x


class _SE(nn.Layer):
    def __init__(self, c, r=4):
        super().__init__()
        self.pool = nn.AdaptiveAvgPool2D(1)
        self.fc1 = nn.Conv2D(c, _div8(c // r), 1)
        self.fc2 = nn.Conv2D(_div8(c // r), c, 1)

    def forward(self, x):
        s = torch.relu(self.fc1(self.pool(x)))
        return x * nn.functional.hardsigmoid(self.fc2(s))


class _MBV3Block(nn.Layer):
    def __init__(self, cin, k, exp, cout, se, act, s):
        super().__init__()
        self.use_res = s == 1 and cin == cout
        layers = [] if exp == cin else [_cbr(cin, exp, 1, act=act)]
        layers.append(_cbr(exp, exp, k, s, k // 2, groups=exp, act=act))
        if se:
            layers.append(_SE(exp))
        layers += [nn.Conv2D(exp, cout, 1, bias_attr=False), nn.BatchNorm2D(cout)]
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.block(x) if self.use_res else self.block(x)


_MBV3 = {
    "large": ([(3, 16, 16, False, "relu", 1), (3, 64, 24, False, "relu", 2), (3, 72, 24, False, "relu", 1),
               (5, 72, 40, True, "relu", 2), (5, 120, 40, True, "relu", 1), (5, 120, 40, True, "relu", 1),
               (3, 240, 80, False, "hardswish", 2), (3, 200, 80, False, "hardswish", 1),
               (3, 184, 80, False, "hardswish", 1), (3, 184, 80, False, "hardswish", 1),
               (3, 480, 112, True, "hardswish", 1), (3, 672, 112, True, "hardswish", 1),
               (5, 672, 160, True, "hardswish", 2), (5, 960, 160, True, "hardswish", 1),
               (5, 960, 160, True, "hardswish", 1)], 960, 1280),
    "small": ([(3, 16, 16, True, "relu", 2), (3, 72, 24, False, "relu", 2), (3, 88, 24, False, "relu", 1),
               (5, 96, 40, True, "hardswish", 2), (5, 240, 40, True, "hardswish", 1),
               (5, 240, 40, True, "hardswish", 1), (5, 120, 48, True, "hardswish", 1),
               (5, 144, 48, True, "hardswish", 1), (5, 288, 96, True, "hardswish", 2),
               (5, 576, 96, True, "hardswish", 1), (5, 576, 96, True, "hardswish", 1)], 576, 1024),
}


class MobileNetV3(nn.Layer):
    def __init__(self, config="large", scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg, last_conv, last_ch = _MBV3[config]
        cin = _div8(16 * scale)
        layers = [_cbr(3, cin, 3, 2, 1, act="hardswish")]
        for k, e, c, se, act, s in cfg:
            cout = _div8(c * scale)
            layers.append(_MBV3Block(cin, k, _div8(e * scale), cout, se, act, s))
            cin = cout
        layers.append(_cbr(cin, _div8(last_conv * scale), 1, act="hardswish"))
        self.features = nn.Sequential(*layers)
        self.num_classes, self.with_pool = num_classes, with_pool
        self.avgpool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(_div8(last_conv * scale), last_ch), nn.Hardswish(),
                                            nn.Dropout(0.2), nn.Linear(last_ch, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        return self.classifier(torch.flatten(x, 1)) if self.num_classes > 0 else x


class MobileNetV3Large(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__("large", scale, num_classes, with_pool)


class MobileNetV3Small(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__("small", scale, num_classes, with_pool)


def mobilenet_v1(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV1(scale, **kw)


def mobilenet_v2(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV2(scale, **kw)


def mobilenet_v3_large(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Large(scale, **kw)


def mobilenet_v3_small(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Small(scale, **kw)


# ----------------------------------------------------------------------------------------- SqueezeNet
class _Fire(nn.Layer):
    def __init__(self, cin, s, e1, e3):
        super().__init__()
        self.squeeze = nn.Sequential(nn.Conv2D(cin, s, 1), nn.ReLU())
        self.e1 = nn.Sequential(nn.Conv2D(s, e1, 1), nn.ReLU())
        self.e3 = nn.Sequential(nn.Conv2D(s, e3, 3, padding=1), nn.ReLU())

    def forward(self, x):
        x = self.squeeze(x)
        return torch.cat([self.e1(x), self.e3(x)], 1)


class SqueezeNet(nn.Layer):
    def __init__(self, version="1.1", num_classes=1000, with_pool=True):
        super().__init__()
        if version == "1.0":
            f = [nn.Conv2D(3, 96, 7, 2), nn.ReLU(), nn.MaxPool2D(3, 2), _Fire(96, 16, 64, 64),
                 _Fire(128, 16, 64, 64), _Fire(128, 32, 128, 128), nn.MaxPool2D(3, 2),
                 _Fire(256, 32, 128, 128), _Fire(256, 48, 192, 192), _Fire(384, 48, 192, 192),
                 _Fire(384, 64, 256, 256), nn.MaxPool2D(3, 2), _Fire(512, 64, 256, 256)]
        else:
            f = [nn.Conv2D(3, 64, 3, 2), nn.ReLU(), nn.MaxPool2D(3, 2), _Fire(64, 16, 64, 64),
                 _Fire(128, 16, 64, 64), nn.MaxPool2D(3, 2), _Fire(128, 32, 128, 128),
                 _Fire(256, 32, 128, 128), nn.MaxPool2D(3, 2), _Fire(256, 48, 192, 192),
                 _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), _Fire(512, 64, 256, 256)]
        self.features = nn.Sequential(*f)
        self.num_classes, self.with_pool = num_classes, with_pool
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.5), nn.Conv2D(512, num_classes, 1), nn.ReLU())
        self.pool = nn.AdaptiveAvgPool2D(1)

    def forward(self, x):
        x = self.features(x)
        if self.num_classes > 0:
            x = self.classifier(x)
        if self.with_pool:
            x = self.pool(x)
        return torch.flatten(x, 1) if self.num_classes > 0 else x


def squeezenet1_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return SqueezeNet("1.0", **kw)


def squeezenet1_1(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return SqueezeNet("1.1", **kw)


# ----------------------------------------------------------------------------------------- ShuffleNetV2
def _channel_shuffle(x, groups):
    b, c, h, w = x.shape
    return x.reshape(b, groups, c // groups, h, w).transpose(1, 2).reshape(b, c, h, w)


class _ShuffleUnit(nn.Layer):
    def __init__(self, cin, cout, stride, act="relu"):
        super().__init__()
        self.stride = stride
        branch = cout // 2
        if stride > 1:
            self.b1 = nn.Sequential(_cbr(cin, cin, 3, stride, 1, groups=cin, act=None), _cbr(cin, branch, 1, act=act))
        b2_in = cin if stride > 1 else branch
        self.b2 = nn.Sequential(_cbr(b2_in, branch, 1, act=act), _cbr(branch, branch, 3, stride, 1, groups=branch, act=None),
                                _cbr(branch, branch, 1, act=act))

    def forward(self, x):
        if self.stride == 1:
            a, b = x.chunk(2, 1)
            out = torch.cat([a, self.b2(b)], 1)
        else:
            out = torch.cat([self.b1(x), self.b2(x)], 1)
        return _channel_shuffle(out, 2)


class ShuffleNetV2(nn.Layer):
    def __init__(self, scale=1.0, act="relu", num_classes=1000, with_pool=True):
        super().__init__()
        ch = {0.25: [24, 24, 48, 96, 512], 0.33: [24, 32, 64, 128, 512], 0.5: [24, 48, 96, 192, 1024],
              1.0: [24, 116, 232, 464, 1024], 1.5: [24, 176, 352, 704, 1024], 2.0: [24, 244, 488, 976, 2048]}[scale]
        self.conv1 = _cbr(3, ch[0], 3, 2, 1, act=act)
        self.maxpool = nn.MaxPool2D(3, 2, 1)
        layers, cin = [], ch[0]
        for stage, reps in enumerate([4, 8, 4]):
            cout = ch[stage + 1]
            for i in range(reps):
                layers.append(_ShuffleUnit(cin, cout, 2 if i == 0 else 1, act))
                cin = cout
        self.stages = nn.Sequential(*layers)
        self.conv_last = _cbr(cin, ch[-1], 1, act=act)
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(ch[-1], num_classes)

    def forward(self, x):
        x = self.conv_last(self.stages(self.maxpool(self.conv1(x))))
        if self.with_pool:
            x = self.pool(x)
        return self.fc(torch.flatten(x, 1)) if self.num_classes > 0 else x


def shufflenet_v2_x1_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(1.0, **kw)


def shufflenet_v2_x0_5(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(0.5, **kw)


def shufflenet_v2_x2_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(2.0, **kw)


# ----------------------------------------------------------------------------------------- DenseNet
class _DenseLayer(nn.Layer):
    def __init__(self, cin, growth, bn_size, dropout):
        super().__init__()
        self.body = nn.Sequential(nn.BatchNorm2D(cin), nn.ReLU(), nn.Conv2D(cin, bn_size * growth, 1, bias_attr=False),
                                  nn.BatchNorm2D(bn_size * growth), nn.ReLU(),
                                  nn.Conv2D(bn_size * growth, growth, 3, padding=1, bias_attr=False))
        self.dropout = nn.Dropout(dropout) if dropout else None

    def forward(self, x):
        y = self.body(x)
        if self.dropout is not None:
            y = self.dropout(y)
        return torch.cat([x, y], 1)


class DenseNet(nn.Layer):
    def __init__(self, layers=121, bn_size=4, dropout=0.0, num_classes=1000, with_pool=True):
        super().__init__()
        growth, init, blocks = {121: (32, 64, [6, 12, 24, 16]), 161: (48, 96, [6, 12, 36, 24]),
                                169: (32, 64, [6, 12, 32, 32]), 201: (32, 64, [6, 12, 48, 32]),
                                264: (32, 64, [6, 12, 64, 48])}[layers]
        f = [nn.Conv2D(3, init, 7, 2, 3, bias_attr=False), nn.BatchNorm2D(init), nn.ReLU(), nn.MaxPool2D(3, 2, 1)]
        c = init
        for i, n in enumerate(blocks):
            for _ in range(n):
                f.append(_DenseLayer(c, growth, bn_size, dropout))
                c += growth
            if i != len(blocks) - 1:
                f += [nn.BatchNorm2D(c), nn.ReLU(), nn.Conv2D(c, c // 2, 1, bias_attr=False), nn.AvgPool2D(2, 2)]
                c //= 2
        f += [nn.BatchNorm2D(c), nn.ReLU()]
        self.features = nn.Sequential(*f)
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.out = nn.Linear(c, num_classes)

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool(x)
        return self.out(torch.flatten(x, 1)) if self.num_classes > 0 else x


def densenet121(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(121, **kw)


def densenet169(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(169, **kw)


def densenet201(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(201, **kw)


def densenet161(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(161, **kw)


def densenet264(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(264, **kw)


def shufflenet_v2_x0_25(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(0.25, **kw)


def shufflenet_v2_x0_33(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(0.33, **kw)


def shufflenet_v2_x1_5(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(1.5, **kw)


def shufflenet_v2_swish(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(1.0, act="swish", **kw)


# ----------------------------------------------------------------------------------------- GoogLeNet
class _Inception(nn.Layer):
    """GoogLeNet inception module (reference `vision/models/googlenet.py`): 1×1 | 1×1→3×3 |
    1×1→5×5 | pool→1×1 branches concatenated on channels."""

    def __init__(self, cin, c1, c3r, c3, c5r, c5, proj):
        super().__init__()
        self.b1 = _cbr(cin, c1, 1)
        self.b2 = nn.Sequential(_cbr(cin, c3r, 1), _cbr(c3r, c3, 3, 1, 1))
        self.b3 = nn.Sequential(_cbr(cin, c5r, 1), _cbr(c5r, c5, 5, 1, 2))
        self.b4 = nn.Sequential(nn.MaxPool2D(3, 1, 1), _cbr(cin, proj, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b2(x), self.b3(x), self.b4(x)], 1)


class GoogLeNet(nn.Layer):
    """Reference `python/paddle/vision/models/googlenet.py` (returns (out, aux1, aux2) like the
    reference: the two auxiliary heads read the 4a / 4d inception outputs)."""

    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.stem = nn.Sequential(_cbr(3, 64, 7, 2, 3), nn.MaxPool2D(3, 2, 1), _cbr(64, 64, 1),
                                  _cbr(64, 192, 3, 1, 1), nn.MaxPool2D(3, 2, 1))
        self.i3 = nn.Sequential(_Inception(192, 64, 96, 128, 16, 32, 32),
                                _Inception(256, 128, 128, 192, 32, 96, 64), nn.MaxPool2D(3, 2, 1))
        self.i4a = _Inception(480, 192, 96, 208, 16, 48, 64)
        self.i4bcd = nn.Sequential(_Inception(512, 160, 112, 224, 24, 64, 64),
                                   _Inception(512, 128, 128, 256, 24, 64, 64),
                                   _Inception(512, 112, 144, 288, 32, 64, 64))
        self.i4e = nn.Sequential(_Inception(528, 256, 160, 320, 32, 128, 128), nn.MaxPool2D(3, 2, 1))
        self.i5 = nn.Sequential(_Inception(832, 256, 160, 320, 32, 128, 128),
                                _Inception(832, 384, 192, 384, 48, 128, 128))
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.4)
            self.fc = nn.Linear(1024, num_classes)
            self.aux1 = nn.Sequential(nn.AdaptiveAvgPool2D(4), _cbr(512, 128, 1), nn.Flatten(),
                                      nn.Linear(2048, 1024), nn.ReLU(), nn.Dropout(0.7),
                                      nn.Linear(1024, num_classes))
            self.aux2 = nn.Sequential(nn.AdaptiveAvgPool2D(4), _cbr(528, 128, 1), nn.Flatten(),
                                      nn.Linear(2048, 1024), nn.ReLU(), nn.Dropout(0.7),
                                      nn.Linear(1024, num_classes))

    def forward(self, x):
        x = self.i3(self.stem(x))
        a = self.i4a(x)
        d = self.i4bcd(a)
        x = self.i5(self.i4e(d))
        if self.with_pool:
            x = self.pool(x)
        if self.num_classes <= 0:
            return x
        out = self.fc(self.dropout(torch.flatten(x, 1)))
        return out, self.aux1(a), self.aux2(d)


def googlenet(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return GoogLeNet(**kw)


# ----------------------------------------------------------------------------------------- InceptionV3
class _IncA(nn.Layer):
    def __init__(self, cin, pool_feat):
        super().__init__()
        self.b1 = _cbr(cin, 64, 1)
        self.b5 = nn.Sequential(_cbr(cin, 48, 1), _cbr(48, 64, 5, 1, 2))
        self.b3 = nn.Sequential(_cbr(cin, 64, 1), _cbr(64, 96, 3, 1, 1), _cbr(96, 96, 3, 1, 1))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1), _cbr(cin, pool_feat, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b5(x), self.b3(x), self.bp(x)], 1)


class _IncB(nn.Layer):  # grid reduction 35 -> 17
    def __init__(self, cin):
        super().__init__()
        self.b3 = _cbr(cin, 384, 3, 2)
        self.b3d = nn.Sequential(_cbr(cin, 64, 1), _cbr(64, 96, 3, 1, 1), _cbr(96, 96, 3, 2))
        self.pool = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return torch.cat([self.b3(x), self.b3d(x), self.pool(x)], 1)


def _cbr_hw(cin, cout, kh, kw, ph, pw):
    return nn.Sequential(nn.Conv2D(cin, cout, (kh, kw), 1, (ph, pw), bias_attr=False),
                         nn.BatchNorm2D(cout), nn.ReLU())


class _IncC(nn.Layer):  # factorised 7x7 (17x17 grid)
    def __init__(self, cin, c7):
        super().__init__()
        self.b1 = _cbr(cin, 192, 1)
        self.b7 = nn.Sequential(_cbr(cin, c7, 1), _cbr_hw(c7, c7, 1, 7, 0, 3), _cbr_hw(c7, 192, 7, 1, 3, 0))
        self.b7d = nn.Sequential(_cbr(cin, c7, 1), _cbr_hw(c7, c7, 7, 1, 3, 0), _cbr_hw(c7, c7, 1, 7, 0, 3),
                                 _cbr_hw(c7, c7, 7, 1, 3, 0), _cbr_hw(c7, 192, 1, 7, 0, 3))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1), _cbr(cin, 192, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b7(x), self.b7d(x), self.bp(x)], 1)


class _IncD(nn.Layer):  # grid reduction 17 -> 8
    def __init__(self, cin):
        super().__init__()
        self.b3 = nn.Sequential(_cbr(cin, 192, 1), _cbr(192, 320, 3, 2))
        self.b7 = nn.Sequential(_cbr(cin, 192, 1), _cbr_hw(192, 192, 1, 7, 0, 3),
                                _cbr_hw(192, 192, 7, 1, 3, 0), _cbr(192, 192, 3, 2))
        self.pool = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return torch.cat([self.b3(x), self.b7(x), self.pool(x)], 1)


class _IncE(nn.Layer):  # expanded filter bank (8x8 grid)
    def __init__(self, cin):
        super().__init__()
        self.b1 = _cbr(cin, 320, 1)
        self.b3 = _cbr(cin, 384, 1)
        self.b3a, self.b3b = _cbr_hw(384, 384, 1, 3, 0, 1), _cbr_hw(384, 384, 3, 1, 1, 0)
        self.b3d = nn.Sequential(_cbr(cin, 448, 1), _cbr(448, 384, 3, 1, 1))
        self.b3da, self.b3db = _cbr_hw(384, 384, 1, 3, 0, 1), _cbr_hw(384, 384, 3, 1, 1, 0)
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1), _cbr(cin, 192, 1))

    def forward(self, x):
        a = self.b3(x)
        d = self.b3d(x)
        return torch.cat([self.b1(x), self.b3a(a), self.b3b(a), self.b3da(d), self.b3db(d), self.bp(x)], 1)


class InceptionV3(nn.Layer):
    """Reference `python/paddle/vision/models/inceptionv3.py` (299×299 inputs)."""

    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.stem = nn.Sequential(_cbr(3, 32, 3, 2), _cbr(32, 32, 3), _cbr(32, 64, 3, 1, 1),
                                  nn.MaxPool2D(3, 2), _cbr(64, 80, 1), _cbr(80, 192, 3), nn.MaxPool2D(3, 2))
        self.blocks = nn.Sequential(_IncA(192, 32), _IncA(256, 64), _IncA(288, 64), _IncB(288),
                                    _IncC(768, 128), _IncC(768, 160), _IncC(768, 160), _IncC(768, 192),
                                    _IncD(768), _IncE(1280), _IncE(2048))
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.2)
            self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        if self.with_pool:
            x = self.pool(x)
        if self.num_classes <= 0:
            return x
        return self.fc(self.dropout(torch.flatten(x, 1)))


def inception_v3(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return InceptionV3(**kw)

"""``paddle.vision`` (reference `python/paddle/vision/`): models, transforms, datasets, ops."""
from . import models  # noqa: F401
from . import transforms  # noqa: F401
from . import datasets  # noqa: F401
from . import ops  # noqa: F401
from .models import (LeNet, AlexNet, VGG, ResNet, MobileNetV1, MobileNetV2, MobileNetV3Small,  # noqa: F401
                     MobileNetV3Large, SqueezeNet, ShuffleNetV2, DenseNet, resnet18, resnet34,
                     resnet50, resnet101, resnet152, vgg11, vgg13, vgg16, vgg19, mobilenet_v1,
                     mobilenet_v2, mobilenet_v3_small, mobilenet_v3_large, alexnet, squeezenet1_0,
                     squeezenet1_1, densenet121, shufflenet_v2_x1_0, wide_resnet50_2,
                     resnext50_32x4d)

_BACKEND = ["cv2"]


def set_image_backend(backend):
    _BACKEND[0] = backend


def get_image_backend():
    return _BACKEND[0]


def image_load(path, backend=None):
    from .datasets import _load_image
    return _load_image(path)

from .vgg16 import VGG16, VGG16Runtime, VGG16_LAYER_NAMES, VGG16_SPECS, LayerSpec

__all__ = ["VGG16", "VGG16Runtime", "VGG16_LAYER_NAMES", "VGG16_SPECS", "LayerSpec"]

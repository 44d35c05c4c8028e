"""Model zoo: the reference's linear regression, MNIST MLP, ResNet-50, BERT-base, GPT-2-medium."""
from .resnet import ResNet, ResNet50, ResNet101, ResNet152  # noqa: F401

"""Model zoo (README.md:85-92): GPT-2, VGG-11/13/16, ResNet-32/50/101 (+ siblings)."""
from .model_factory import ModelFactory, get_model, SUPPORTED  # noqa: F401
from .gpt2 import GPT2Config, GPT2LMHeadModel  # noqa: F401

"""Adversary / fault injection (README.md:61: ``from trustworthy_dl.attacks import AdversarialAttacker``)."""
from .adversarial_attacks import AdversarialAttacker, AttackConfig, ATTACK_TYPES  # noqa: F401

"""Security layer: attack detection, gradient verification, device stage verifier."""
from .attack_detection import AttackDetector, AttackType, AttackDetectionResult  # noqa: F401
from .gradient_verification import GradientVerifier  # noqa: F401

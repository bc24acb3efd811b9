"""trustworthy_dl — MI355X-native trustworthy model-parallel training.

Public API (README.md:57-82 of the reference): DistributedTrainer, TrustManager, AttackDetector,
GradientVerifier, AdversarialAttacker, get_model.
"""
__version__ = "0.1.0"

# before anything touches the GPU: enough HIP hardware queues that the pipeline's pre-posted RCCL
# receives never share a queue with the compute stream (runtime/hwqueues.py)
from .runtime.hwqueues import ensure_hw_queues as _ensure_hw_queues
_ensure_hw_queues()

from .core.trust_manager import TrustManager, NodeStatus  # noqa: F401
from .security.attack_detection import AttackDetector, AttackType  # noqa: F401
from .security.gradient_verification import GradientVerifier  # noqa: F401
from .models import get_model, ModelFactory  # noqa: F401


def __getattr__(name):  # lazy: trainer/attacks pull in the engine
    if name in ("DistributedTrainer", "TrainingConfig", "TrainingState", "NodeConfig"):
        from .core import distributed_trainer as m
        return getattr(m, name)
    if name in ("AdversarialAttacker", "AttackConfig"):
        from .attacks import adversarial_attacks as m
        return getattr(m, name)
    raise AttributeError(name)

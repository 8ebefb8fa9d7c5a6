"""Mirror of /root/reference/models/__init__.py:1-3 (imports cleanly: SURVEY.md finding 4)."""
from . import adversarial, builder, detectors  # noqa: F401

__all__ = ["adversarial", "detectors", "builder"]

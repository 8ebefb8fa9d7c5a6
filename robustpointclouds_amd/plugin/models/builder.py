"""Mirror of models/builder.py:6-11: the ADVERSARIES registry and build_adversary."""
try:   # the reference's registry when mmengine is installed
    from mmengine.registry import Registry

    ADVERSARIES = Registry("adversaries", parent=None, scope="models")
except ImportError:   # standalone: this framework's registry
    from robustpointclouds_amd.registry import ADVERSARIES


def build_adversary(cfg):
    """Build an adversary from its config dict (models/builder.py:8-11)."""
    return ADVERSARIES.build(cfg)

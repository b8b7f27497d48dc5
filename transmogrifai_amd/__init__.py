"""transmogrifai_amd -- an MI355X-native AutoML engine for structured data."""
__version__ = "0.1.0"


def register_function(fn=None, name=None):
    """Register a user function (feature extract / predicate) so checkpoints naming it can restore it.
    Checkpoints never import modules; see :func:`transmogrifai_amd.stages.generator.register_function`."""
    from .stages.generator import register_function as _r
    return _r(fn, name)

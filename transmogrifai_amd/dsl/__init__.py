"""Feature DSL: typed methods available on features (``core/.../dsl/Rich*Feature.scala``).

Methods are registered per feature type and resolved dynamically by ``FeatureLike.__getattr__``, so
``age.fill_missing_with_mean().z_normalize()``, ``sex.pivot()``, ``label.sanity_check(vec)`` work as in
the reference DSL. Collection helpers (``transmogrify``, ``combine``) are module-level functions.
"""
_REGISTRY = {}
_loaded = False


def register(types, name):
    def deco(fn):
        for t in (types if isinstance(types, (list, tuple)) else [types]):
            _REGISTRY.setdefault(name, []).append((t, fn))
        return fn
    return deco


def _ensure():
    global _loaded
    if not _loaded:
        _loaded = True
        from . import core  # noqa: F401


def lookup(wtype, name):
    if name.startswith("__"):
        return None
    _ensure()
    # the most specific registration wins (Date.vectorize is the date vectorizer even though a Date is an
    # Integral): the matching type closest to ``wtype`` in its MRO, the first registered among equals
    best, best_d = None, None
    mro = wtype.__mro__
    for t, fn in _REGISTRY.get(name, []):
        if issubclass(wtype, t):
            d = mro.index(t) if t in mro else len(mro)
            if best_d is None or d < best_d:
                best, best_d = fn, d
    return best


def binary_op(a, b, op, reverse=False):
    _ensure()
    from .core import _binary_op
    return _binary_op(a, b, op, reverse)


def transmogrify(features, label=None, defaults=None):
    from ..stages.feature.transmogrifier import TransmogrifierDefaults, transmogrify_combined
    return transmogrify_combined(list(features), label, defaults or TransmogrifierDefaults)


def auto_transform(features, label=None, defaults=None):
    """``RichFeaturesCollection.autoTransform`` (RichFeaturesCollection.scala:79): alias of :func:`transmogrify`."""
    return transmogrify(features, label, defaults)


def combine(*vectors):
    from ..stages.feature.vectorizers import VectorsCombiner
    vs = []
    for v in vectors:
        vs.extend(v if isinstance(v, (list, tuple)) else [v])
    return VectorsCombiner().set_input(vs).get_output()

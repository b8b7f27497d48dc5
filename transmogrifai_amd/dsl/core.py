"""DSL method implementations (``RichNumericFeature``, ``RichTextFeature``, ``RichDateFeature``,
``RichListFeature``, ``RichSetFeature``, ``RichMapFeature``, ``RichVectorFeature``, ``RichLocationFeature``)."""
from __future__ import annotations

from typing import Callable, Optional, Sequence

from ..features import types as T
from ..features.feature import FeatureLike
from ..stages.base import BinaryTransformer, UnaryTransformer
from ..stages.feature import math_stages as M
from ..stages.feature import text_stages as TS
from ..stages.feature import vectorizers as V
from ..stages.feature.transmogrifier import TransmogrifierDefaults as D
from . import register

NUM = (T.OPNumeric,)


def _others(f, others):
    return [f] + list(others or [])


# ------------------------------------------------------------------------------------- generic
@register(T.FeatureType, "map")
def _map(self: FeatureLike, fn: Callable, output_type=T.Text, operation_name: str = "map"):
    from ..stages.feature.misc_stages import MapTransformer
    return MapTransformer(fn, output_type, operation_name).set_input(self).get_output()


@register(T.FeatureType, "alias")
def _alias(self, name: str):
    from ..stages.feature.misc_stages import AliasTransformer
    return AliasTransformer(name).set_input(self).get_output()


@register(T.FeatureType, "exists")
def _exists(self, fn: Callable):
    from ..stages.feature.misc_stages import ExistsTransformer
    return ExistsTransformer(fn).set_input(self).get_output()


@register(T.FeatureType, "filter")
def _filter(self, fn: Callable, default=None):
    from ..stages.feature.misc_stages import FilterTransformer
    return FilterTransformer(fn, default).set_input(self).get_output()


@register(T.FeatureType, "replace_with")
def _replace(self, old, new):
    from ..stages.feature.misc_stages import ReplaceTransformer
    return ReplaceTransformer(old_value=old, new_value=new).set_input(self).get_output()


@register(T.FeatureType, "occurs")         # RichFeature.occurs (RichFeature.scala): the same transformer
@register(T.FeatureType, "to_occur")
def _to_occur(self, match_fn: Optional[Callable] = None):
    from ..stages.feature.misc_stages import ToOccurTransformer
    return ToOccurTransformer(match_fn).set_input(self).get_output()


@register(T.Text, "is_substring")
def _substring(self, full: FeatureLike, to_lowercase: bool = True):
    """``self`` is contained in ``full`` (``RichTextFeature.isSubstring``)."""
    from ..stages.feature.misc_stages import SubstringTransformer
    return SubstringTransformer(to_lowercase=to_lowercase).set_input(self, full).get_output()


@register(T.Text, "to_n_gram_similarity")
def _ngram_text(self, other: FeatureLike, n_gram_size: int = 3, to_lowercase: bool = True):
    from ..stages.feature.misc_stages import TextNGramSimilarity
    return TextNGramSimilarity(n_gram_size=n_gram_size, to_lowercase=to_lowercase).set_input(self, other).get_output()


@register(T.MultiPickList, "to_n_gram_similarity")
def _ngram_set(self, other: FeatureLike, n_gram_size: int = 3, to_lowercase: bool = True):
    from ..stages.feature.misc_stages import SetNGramSimilarity
    return SetNGramSimilarity(n_gram_size=n_gram_size, to_lowercase=to_lowercase).set_input(self, other).get_output()


@register(T.MultiPickList, "jaccard_similarity")
def _jaccard(self, other: FeatureLike):
    from ..stages.feature.misc_stages import JaccardSimilarity
    return JaccardSimilarity().set_input(self, other).get_output()


@register(T.Date, "to_time_period")
def _time_period(self, period: str):
    from ..stages.feature.misc_stages import TimePeriodTransformer
    return TimePeriodTransformer(period=period).set_input(self).get_output()


@register(T.DateList, "to_time_period")
def _time_period_list(self, period: str):
    from ..stages.feature.misc_stages import TimePeriodListTransformer
    return TimePeriodListTransformer(period=period).set_input(self).get_output()


@register(T.DateMap, "to_time_period")
def _time_period_map(self, period: str):
    from ..stages.feature.misc_stages import TimePeriodMapTransformer
    return TimePeriodMapTransformer(period=period).set_input(self).get_output()


@register(T.OPMap, "filter_keys")
def _filter_map(self, allow_list_keys=(), block_list_keys=(), clean_keys: bool = False, clean_text: bool = True):
    from ..stages.feature.misc_stages import FilterMap
    return FilterMap(allow_list_keys=list(allow_list_keys), block_list_keys=list(block_list_keys),
                     clean_keys=clean_keys, clean_text=clean_text).set_input(self).get_output()


@register(T.EmailMap, "to_email_domains")
def _email_map(self):
    from ..stages.feature.misc_stages import EmailToPickListMapTransformer
    return EmailToPickListMapTransformer().set_input(self).get_output()


@register(T.URLMap, "to_domains")
def _url_map(self):
    from ..stages.feature.misc_stages import UrlMapToPickListMapTransformer
    return UrlMapToPickListMapTransformer().set_input(self).get_output()


# ------------------------------------------------------------------------------------- numeric
def _binary_op(a, b, op, reverse=False):
    if isinstance(b, FeatureLike):
        x, y = (b, a) if reverse else (a, b)
        return M.BinaryMathTransformer(op).set_input(x, y).get_output()
    return M.ScalarMathTransformer(op, float(b), reverse).set_input(a).get_output()


for _op in ("abs", "ceil", "floor", "round", "exp", "sqrt"):
    def _mk(op):
        def f(self):
            return M.UnaryMathTransformer(op).set_input(self).get_output()
        return f
    register(NUM, _op)(_mk(_op))


@register(NUM, "log")
def _log(self, base: float = 2.718281828459045):
    return M.UnaryMathTransformer("log", base=base).set_input(self).get_output()


@register(NUM, "power")
def _power(self, p: float):
    return M.ScalarMathTransformer("power", p).set_input(self).get_output()


@register(NUM, "round_digits")
def _round_digits(self, digits: int):
    return M.UnaryMathTransformer("roundDigits", digits=digits).set_input(self).get_output()


@register(NUM, "fill_missing_with_mean")
def _fill_mean(self, default: float = 0.0):
    return M.FillMissingWithMean(default_value=default).set_input(self).get_output()


@register(NUM, "z_normalize")
def _znorm(self):
    return M.OpScalarStandardScaler().set_input(self).get_output()


@register(NUM, "to_percentile")
def _pct(self, buckets: int = 100):
    return M.PercentileCalibrator(expected_num_buckets=buckets).set_input(self).get_output()


@register(NUM, "scale")
def _scale(self, scaling_type: str = "Linear", slope: float = 1.0, intercept: float = 0.0):
    return M.ScalerTransformer(scaling_type=scaling_type, slope=slope, intercept=intercept).set_input(self).get_output()


def _scaling_of(scaled):
    st = scaled.origin_stage
    if isinstance(st, M.ScalerTransformer):
        return {k: st.params[k] for k in ("scaling_type", "slope", "intercept")}
    if isinstance(st, (M.OpScalarStandardScaler, M.OpScalarStandardScalerModel)):
        return {}          # linear scaling known after the fit: read from the scaler metadata at transform
    raise ValueError(f"feature '{scaled.name}' was not produced by a scaler (scale() / z_normalize())")


@register(NUM, "descale")
def _descale(self, scaled):
    """Inverse of ``scaled``'s scaling applied to this feature (``RichNumericFeature.descale``)."""
    return M.DescalerTransformer(**_scaling_of(scaled)).set_input(self, scaled).get_output()


def descale_prediction(prediction, scaled):
    """``PredictionDescaler``: a model's prediction back on the scale of the unscaled label."""
    return M.PredictionDescaler(**_scaling_of(scaled)).set_input(prediction, scaled).get_output()


@register(NUM, "bucketize")
def _bucketize(self, splits: Sequence[float], track_nulls: bool = True, track_invalid: bool = False,
               split_inclusion: str = "Left", bucket_labels=None):
    return M.NumericBucketizer(splits=list(splits), track_nulls=track_nulls, track_invalid=track_invalid,
                               split_inclusion=split_inclusion, bucket_labels=bucket_labels).set_input(self).get_output()


@register(NUM, "auto_bucketize")
def _auto_bucketize(self, label: FeatureLike, track_nulls: bool = True, track_invalid: bool = False,
                    min_info_gain: float = 0.01):
    from ..stages.feature.bucketizers import DecisionTreeNumericBucketizer
    return DecisionTreeNumericBucketizer(track_nulls=track_nulls, track_invalid=track_invalid,
                                         min_info_gain=min_info_gain).set_input(label, self).get_output()


@register(T.RealNN, "to_isotonic_calibrated")
def _iso(self, label: FeatureLike, isotonic: bool = True):
    return M.IsotonicRegressionCalibrator(isotonic=isotonic).set_input(label, self).get_output()


@register((T.Real, T.Currency, T.Percent), "vectorize")
def _vec_real(self, fill_value: float = 0.0, fill_with_mean: bool = True, track_nulls: bool = True, others=(),
              label: Optional[FeatureLike] = None, **kw):
    if self.wtype is T.RealNN and not others:
        return V.RealNNVectorizer().set_input(self).get_output()
    st = V.RealVectorizer(track_nulls=track_nulls, fill_value=float(fill_value))
    if fill_with_mean:
        st.set_fill_with_mean()
    return _with_buckets(self, st.set_input(_others(self, others)).get_output(), others, label, kw)


def _with_buckets(self, out, others, label, kw):
    """The label-aware buckets a numeric ``vectorize(label = ...)`` appends (RichNumericFeature.scala:329-336,
    :660-667): ``autoBucketize(label, trackNulls = false, trackInvalid, minInfoGain)`` per feature."""
    if label is None:
        return out
    from ..stages.feature.bucketizers import DecisionTreeNumericBucketizer
    bs = [DecisionTreeNumericBucketizer(track_nulls=False, track_invalid=kw.get("track_invalid", D.TrackInvalid),
                                        min_info_gain=kw.get("min_info_gain", D.MinInfoGain))
          .set_input(label, f).get_output() for f in _others(self, others)]
    return V.VectorsCombiner().set_input([out] + bs).get_output()


@register(T.RealNN, "vectorize")
def _vec_realnn(self, others=(), **kw):
    return V.RealNNVectorizer().set_input(_others(self, others)).get_output()


@register(T.Integral, "vectorize")
def _vec_int(self, fill_value: float = 0.0, fill_with_mode: bool = True, track_nulls: bool = True, others=(),
             label=None, **kw):
    st = V.IntegralVectorizer(track_nulls=track_nulls, fill_value=float(fill_value))
    if fill_with_mode:
        st.set_fill_with_mode()
    return _with_buckets(self, st.set_input(_others(self, others)).get_output(), others, label, kw)


@register(T.Binary, "vectorize")
def _vec_bin(self, fill_value: bool = False, track_nulls: bool = True, others=(), **kw):
    return V.BinaryVectorizer(fill_value=fill_value, track_nulls=track_nulls).set_input(_others(self, others)).get_output()


@register(T.RealNN, "sanity_check")
def _sanity(self, features: FeatureLike, check_sample: float = 1.0, sample_seed: int = 42,
            sample_lower_limit: int = 1000, sample_upper_limit: int = 1_000_000, max_correlation: float = 0.95,
            min_correlation: float = 0.0, min_variance: float = 1e-5, max_cramers_v: float = 0.95,
            remove_bad_features: bool = False, remove_feature_group: bool = True,
            protect_text_shared_hash: bool = False, max_rule_confidence: float = 1.0,
            min_required_rule_support: float = 1.0, correlation_type: str = "pearson",
            feature_feature_corr_level: str = "Computed", categorical_label: Optional[bool] = None,
            max_feature_correlation: float = 0.99, correlation_exclusion: str = "NoExclusion"):
    from ..stages.preparators.sanity_checker import SanityChecker
    st = SanityChecker(check_sample=check_sample, sample_seed=sample_seed, sample_lower_limit=sample_lower_limit,
                       sample_upper_limit=sample_upper_limit, max_correlation=max_correlation,
                       min_correlation=min_correlation, min_variance=min_variance, max_cramers_v=max_cramers_v,
                       remove_bad_features=remove_bad_features, remove_feature_group=remove_feature_group,
                       protect_text_shared_hash=protect_text_shared_hash, max_rule_confidence=max_rule_confidence,
                       min_required_rule_support=min_required_rule_support, correlation_type=correlation_type,
                       feature_feature_corr_level=feature_feature_corr_level, categorical_label=categorical_label,
                       max_feature_correlation=max_feature_correlation, correlation_exclusion=correlation_exclusion)
    return st.set_input(self, features).get_output()


# ---------------------------------------------------------------------------------------- text
@register(T.Text, "pivot")
def _pivot(self, others=(), top_k: int = 20, min_support: int = 10, clean_text: bool = True,
           track_nulls: bool = True, max_pct_cardinality: float = 1.0, unseen_name: str = "OTHER"):
    return V.OpTextPivotVectorizer(top_k=top_k, min_support=min_support, clean_text=clean_text,
                                   track_nulls=track_nulls, max_pct_cardinality=max_pct_cardinality,
                                   unseen_name=unseen_name).set_input(_others(self, others)).get_output()


@register(T.Text, "smart_vectorize")
def _smart(self, max_categorical_cardinality: int = 30, num_hashes: int = 512, track_nulls: bool = True,
           others=(), hash_space_strategy: str = "auto", min_token_length: int = 1, to_lowercase: bool = True,
           prepend_feature_name: bool = True, track_text_len: bool = False, **kw):
    return V.SmartTextVectorizer(max_cardinality=max_categorical_cardinality, num_features=num_hashes,
                                 track_nulls=track_nulls, hash_space_strategy=hash_space_strategy,
                                 min_token_length=min_token_length, to_lowercase=to_lowercase,
                                 prepend_feature_name=prepend_feature_name, track_text_len=track_text_len
                                 ).set_input(_others(self, others)).get_output()


@register(T.Text, "vectorize")
def _vec_text(self, num_terms: int = 512, binary: bool = False, others=(), auto_detect_language: bool = False,
              min_token_length: int = 1, to_lowercase: bool = True, hash_space_strategy: str = "auto",
              prepend_feature_name: bool = True, top_k: int = 20, min_support: int = 10, clean_text: bool = True,
              track_nulls: bool = True, **kw):
    if self.wtype in (T.Text, T.TextArea):
        # RichTextFeature.vectorize (RichTextFeature.scala:135-187): tokenize, hash, then the token lists' text
        # lengths (track_text_len) and null indicators (track_nulls) combined after the hashes
        toks = [TS.TextTokenizer(min_token_length=min_token_length, to_lowercase=to_lowercase)
                .set_input(f).get_output() for f in _others(self, others)]
        hashed = V.OPCollectionHashingVectorizer(num_features=num_terms, binary_freq=binary,
                                                 hash_space_strategy=hash_space_strategy,
                                                 prepend_feature_name=prepend_feature_name).set_input(toks).get_output()
        parts = [hashed]
        if kw.get("track_text_len", False):
            parts.append(TS.TextLenTransformer().set_input(toks).get_output())
        if track_nulls:
            parts.append(TS.TextListNullTransformer().set_input(toks).get_output())
        return parts[0] if len(parts) == 1 else V.VectorsCombiner().set_input(parts).get_output()
    return _pivot(self, others, top_k, min_support, clean_text, track_nulls)


@register(T.Text, "tokenize")
def _tokenize(self, to_lowercase: bool = True, min_token_length: int = 1, strip_html: bool = False, **kw):
    return TS.TextTokenizer(to_lowercase=to_lowercase, min_token_length=min_token_length,
                            strip_html=strip_html).set_input(self).get_output()


@register(T.Email, "to_email_domain")
def _email_domain(self):
    return TS.TextMapTransformer("EmailDomainToPickList", T.Text).set_input(self).get_output()


@register(T.Email, "to_email_prefix")
def _email_prefix(self):
    return TS.TextMapTransformer("EmailPrefixToText", T.Text).set_input(self).get_output()


@register(T.Email, "is_valid_email")
def _valid_email(self):
    return TS.ValidEmailTransformer().set_input(self).get_output()


@register(T.URL, "to_domain")
def _url_domain(self):
    return TS.TextMapTransformer("URLDomainToText", T.Text).set_input(self).get_output()


@register(T.URL, "to_protocol")
def _url_proto(self):
    return TS.TextMapTransformer("URLProtocolToText", T.Text).set_input(self).get_output()


@register(T.Phone, "is_valid_phone_default_country")
def _phone_valid(self, default_region: str = "US", is_strict: bool = False):
    return TS.PhoneValidator(default_region=default_region, strict=is_strict).set_input(self).get_output()


@register(T.Base64, "detect_mime_types")
def _mime(self, type_hint: Optional[str] = None):
    """``RichBase64Feature.detectMimeTypes`` (RichTextFeature.scala:712-731)."""
    from ..stages.feature.nlp_stages import MimeTypeDetector
    return MimeTypeDetector(type_hint=type_hint or "").set_input(self).get_output()


# The typed text features vectorize through what they carry, not their raw strings (``RichTextFeature.scala``):
# an email / URL by its domain (:617-632, :667-682; invalid URLs are empty), base64 content by its detected MIME
# type (:712-729), each pivoted; a phone number by its validity as a binary (:566-575).
@register(T.Email, "vectorize")
def _vec_email(self, top_k: int = 20, clean_text: bool = True, min_support: int = 10, track_nulls: bool = True,
               others=(), max_pct_cardinality: float = 1.0, **kw):
    doms = [TS.TextMapTransformer("EmailDomainToPickList", T.PickList).set_input(f).get_output()
            for f in _others(self, others)]
    return _pivot(doms[0], doms[1:], top_k, min_support, clean_text, track_nulls, max_pct_cardinality)


@register(T.URL, "vectorize")
def _vec_url(self, top_k: int = 20, clean_text: bool = True, min_support: int = 10, track_nulls: bool = True,
             others=(), max_pct_cardinality: float = 1.0, **kw):
    doms = [TS.TextMapTransformer("URLDomainToPickList", T.PickList).set_input(f).get_output()
            for f in _others(self, others)]
    return _pivot(doms[0], doms[1:], top_k, min_support, clean_text, track_nulls, max_pct_cardinality)


@register(T.Base64, "vectorize")
def _vec_base64(self, top_k: int = 20, min_support: int = 10, clean_text: bool = True, track_nulls: bool = True,
                type_hint: Optional[str] = None, others=(), max_pct_cardinality: float = 1.0, **kw):
    mts = [_mime(f, type_hint) for f in _others(self, others)]
    return _pivot(mts[0], mts[1:], top_k, min_support, clean_text, track_nulls, max_pct_cardinality)


@register(T.Phone, "vectorize")
def _vec_phone(self, default_region: str = "US", is_strict: bool = False, track_nulls: bool = True,
               fill_value: bool = False, others=(), **kw):
    valid = [_phone_valid(f, default_region, is_strict) for f in _others(self, others)]
    return V.BinaryVectorizer(fill_value=fill_value, track_nulls=track_nulls).set_input(valid).get_output()


@register(T.Text, "text_len")
def _text_len(self, others=()):
    return TS.TextLenTransformer().set_input(_others(self, others)).get_output()


@register(T.Text, "indexed")
def _indexed(self, unseen_name: str = "UnseenLabel", handle_invalid: str = "NoFilter"):
    from ..stages.feature.indexers import OpStringIndexerNoFilter
    return OpStringIndexerNoFilter(unseen_name=unseen_name).set_input(self).get_output()


# --------------------------------------------------------------------------------- collections
@register(T.TextList, "tf")
def _tf(self, num_terms: int = 512, binary: bool = False):
    return TS.OpHashingTF(num_features=num_terms, binary=binary).set_input(self).get_output()


@register(T.TextList, "tfidf")
def _tfidf(self, num_terms: int = 512, binary: bool = False, min_doc_freq: int = 0):
    return TS.IDF(min_doc_freq=min_doc_freq).set_input(_tf(self, num_terms, binary)).get_output()


@register(T.TextList, "vectorize")
def _vec_tl(self, num_terms: int = 512, binary: bool = False, min_doc_freq: int = 0, others=()):
    vs = [_tfidf(f, num_terms, binary, min_doc_freq) for f in _others(self, others)]
    return V.VectorsCombiner().set_input(vs).get_output() if len(vs) > 1 else vs[0]


@register((T.OPList, T.OPSet, T.OPMap), "hash_vectorize")
def _hash_vec(self, num_terms: int = 512, binary: bool = False, others=()):
    return V.OPCollectionHashingVectorizer(num_features=num_terms, binary_freq=binary).set_input(
        _others(self, others)).get_output()


@register(T.MultiPickList, "vectorize")
def _vec_mpl(self, top_k: int = 20, min_support: int = 10, clean_text: bool = True, track_nulls: bool = True,
             others=(), **kw):
    return V.OpSetVectorizer(top_k=top_k, min_support=min_support, clean_text=clean_text,
                             track_nulls=track_nulls).set_input(_others(self, others)).get_output()


@register(T.MultiPickList, "pivot")
def _pivot_mpl(self, **kw):
    return _vec_mpl(self, **kw)


@register((T.Date, T.DateList), "vectorize")
def _vec_date(self, date_list_pivot: str = "SinceLast", reference_date=None, track_nulls: bool = True,
              circular_date_reps=D.CircularDateRepresentations, others=()):
    fs = _others(self, others)
    since = V.DateListVectorizer(pivot=date_list_pivot, reference_date=reference_date,
                                 track_nulls=track_nulls).set_input(fs).get_output()
    if issubclass(self.wtype, T.DateList) or not circular_date_reps:
        return since
    circ = [V.DateToUnitCircleTransformer(time_period=p).set_input(fs).get_output() for p in circular_date_reps]
    return V.VectorsCombiner().set_input(circ + [since]).get_output()


@register(T.Date, "to_unit_circle")
def _unit_circle(self, time_period: str = "HourOfDay", others=()):
    return V.DateToUnitCircleTransformer(time_period=time_period).set_input(_others(self, others)).get_output()


@register(T.Geolocation, "vectorize")
def _vec_geo(self, fill_with_mean: bool = True, track_nulls: bool = True, others=(), **kw):
    return V.GeolocationVectorizer(fill_with_constant=not fill_with_mean, track_nulls=track_nulls).set_input(
        _others(self, others)).get_output()


@register((T.RealMap, T.IntegralMap), "auto_bucketize")
def _auto_bucketize_map(self, label: FeatureLike, track_nulls: bool = True, track_invalid: bool = False,
                        min_info_gain: float = 0.01, clean_keys: bool = False, allow_list_keys=(),
                        block_list_keys=()):
    """``RichRealMapFeature.autoBucketize`` / ``RichIntegralMapFeature.autoBucketize``: one label-aware tree per
    map key (DecisionTreeNumericMapBucketizer)."""
    from ..stages.feature.bucketizers import DecisionTreeNumericMapBucketizer
    return DecisionTreeNumericMapBucketizer(
        track_nulls=track_nulls, track_invalid=track_invalid, min_info_gain=min_info_gain, clean_keys=clean_keys,
        allow_keys=list(allow_list_keys) or None, block_keys=list(block_list_keys) or None
    ).set_input(label, self).get_output()


@register([T.TextMap, T.TextAreaMap], "vectorize")
def _vec_text_map_dispatch(self, *a, **kw):
    # the converted map types (EmailMap, URLMap, PhoneMap, Base64Map, ...) keep their own RichMapFeature vectorize
    if self.wtype in (T.TextMap, T.TextAreaMap):
        return _vec_text_map(self, *a, **kw)
    return _vec_map(self, *a, **kw)


def _vec_text_map(self, clean_text: bool = True, clean_keys: bool = D.CleanKeys,
                  should_prepend_feature_name: bool = D.PrependFeatureName, allow_list_keys=(), block_list_keys=(),
                  others=(), track_nulls: bool = D.TrackNulls, track_text_len: bool = D.TrackTextLen,
                  num_hashes: int = D.DefaultNumOfFeatures, hash_space_strategy: str = D.HashSpaceStrategy, **kw):
    """``RichTextMapFeature.vectorize`` (RichMapFeature.scala:188-250): text maps are HASHED (every value's tokens of
    every key into one shared space), with per-key text lengths / null indicators from the raw maps."""
    from ..stages.feature.maps import TextMapHashingVectorizer, TextMapLenEstimator, TextMapNullEstimator
    fs = _others(self, others)
    hashed = TextMapHashingVectorizer(num_features=int(kw.get("num_terms", num_hashes)), clean_keys=clean_keys,
                                      clean_text=clean_text, prepend_feature_name=should_prepend_feature_name,
                                      allow_keys=list(allow_list_keys) or None,
                                      block_keys=list(block_list_keys) or None).set_input(fs).get_output()
    parts = [hashed]
    if track_text_len:
        parts.append(TextMapLenEstimator(clean_keys=clean_keys).set_input(fs).get_output())
    if track_nulls:
        parts.append(TextMapNullEstimator(clean_keys=clean_keys).set_input(fs).get_output())
    return parts[0] if len(parts) == 1 else V.VectorsCombiner().set_input(parts).get_output()


@register(T.OPMap, "vectorize")
def _vec_map(self, others=(), **kw):
    """``RichMapFeature.vectorize`` (RichMapFeature.scala): Transmogrifier defaults, overridable by name
    (``default_value``, ``fill_with_mean`` / ``fill_with_mode``, ``clean_keys``, ``top_k``, ``min_support``,
    ``track_nulls``, ``white_list_keys`` / ``black_list_keys``, ...)."""
    from ..stages.feature.maps import map_vectorize
    return map_vectorize(self.wtype, _others(self, others), None, D, **kw)[0]


@register(T.PhoneMap, "is_valid_phone_default_country_map")
def _phone_map_valid(self, is_strict: bool = False, default_region: str = "US"):
    """``RichPhoneMapFeature.isValidPhoneDefaultCountryMap`` (RichMapFeature.scala:979-993) -> BinaryMap."""
    from ..stages.feature.nlp_stages import IsValidPhoneMapDefaultCountry
    return IsValidPhoneMapDefaultCountry(default_region=default_region, strict=is_strict).set_input(self).get_output()


@register(T.Base64Map, "detect_mime_types")
def _mime_map(self, type_hint: Optional[str] = None):
    """``RichBase64MapFeature.detectMimeTypes`` (RichMapFeature.scala:128-132) -> PickListMap."""
    from ..stages.feature.nlp_stages import MimeTypeMapDetector
    return MimeTypeMapDetector(type_hint=type_hint or "").set_input(self).get_output()


@register(T.OPVector, "drop_indices_by")
def _drop_indices_by(self, match_fn: Callable):
    from ..stages.feature.vector_stages import DropIndicesByTransformer
    return DropIndicesByTransformer(match_fn).set_input(self).get_output()


@register(T.OPVector, "filter_min_variance")
def _min_var(self, min_variance: float = 1e-5, remove_bad_features: bool = False):
    from ..stages.preparators.min_variance import MinVarianceFilter
    return MinVarianceFilter(min_variance=min_variance, remove_bad_features=remove_bad_features).set_input(
        self).get_output()


@register(T.OPVector, "combine")
def _combine(self, *others):
    return V.VectorsCombiner().set_input([self] + list(others)).get_output()


# ----------------------------------------------------------------- NLP / type detection entry points
@register(T.Text, "tokenize_regex")
def _tokenize_regex(self, pattern: str, group: int = -1, min_token_length: int = 1, to_lowercase: bool = True):
    """``RichTextFeature.tokenizeRegex`` (``RichTextFeature.scala:375-392``)."""
    return TS.TextRegexTokenizer(pattern=pattern, group=group, min_token_length=min_token_length,
                                 to_lowercase=to_lowercase).set_input(self).get_output()


@register(T.Text, "detect_languages")
def _detect_languages(self):
    """``RichTextFeature.detectLanguages`` -> RealMap of language confidences."""
    from ..stages.feature.nlp_stages import LangDetector
    return LangDetector().set_input(self).get_output()


@register(T.Text, "recognize_entities")
def _recognize_entities(self):
    """``RichTextFeature.recognizeEntities`` -> MultiPickListMap of entity type -> tokens."""
    from ..stages.feature.nlp_stages import NameEntityRecognizer
    return NameEntityRecognizer().set_input(self).get_output()


@register(T.Text, "identify_if_human_name")
def _identify_human_name(self, threshold: float = 0.5):
    """``RichTextFeature.identifyIfHumanName(threshold)`` -> NameStats (``RichTextFeature.scala:456-457``)."""
    from ..stages.feature.nlp_stages import HumanNameDetector
    return HumanNameDetector(threshold=threshold).set_input(self).get_output()


@register(T.Phone, "parse_phone_default_country")
def _parse_phone_default(self, default_region: str = "US"):
    """``RichPhoneFeature.parsePhoneDefaultCountry`` -> normalised Phone."""
    from ..stages.feature.nlp_stages import ParsePhoneNumber
    return ParsePhoneNumber(default_region=default_region).set_input(self).get_output()


@register(T.Phone, "parse_phone")
def _parse_phone(self, default_region: str = "US"):
    return _parse_phone_default(self, default_region)


@register(T.URL, "is_valid_url")
def _is_valid_url(self):
    return TS.ValidUrlTransformer().set_input(self).get_output()


@register(T.TextList, "remove_stop_words")
def _remove_stop_words(self, stop_words=None, case_sensitive: bool = False):
    """``RichListFeature.removeStopWords`` (``RichListFeature.scala:94-166``)."""
    from ..stages.feature.nlp_stages import OpStopWordsRemover
    return OpStopWordsRemover(stop_words=stop_words, case_sensitive=case_sensitive).set_input(self).get_output()


@register(T.TextList, "ngram")
def _ngram(self, n: int = 2):
    from ..stages.feature.nlp_stages import OpNGram
    return OpNGram(n=n).set_input(self).get_output()


@register(T.TextList, "count_vec")
def _count_vec(self, vocab_size: int = 1 << 18, min_df: float = 1.0, min_tf: float = 1.0, binary: bool = False):
    from ..stages.feature.nlp_stages import OpCountVectorizer
    return OpCountVectorizer(vocab_size=vocab_size, min_df=min_df, min_tf=min_tf,
                             binary=binary).set_input(self).get_output()


@register(T.TextList, "word2vec")
def _word2vec(self, vector_size: int = 100, window_size: int = 5, min_count: int = 5, max_iter: int = 1,
              step_size: float = 0.025, **kw):
    from ..stages.feature.nlp_stages import OpWord2Vec
    return OpWord2Vec(vector_size=vector_size, window_size=window_size, min_count=min_count, max_iter=max_iter,
                      step_size=step_size, **kw).set_input(self).get_output()


@register(T.OPVector, "lda")
def _lda(self, k: int = 10, max_iter: int = 20, seed: int = 0, **kw):
    """``RichVectorFeature.lda`` (``RichVectorFeature.scala:115``)."""
    from ..stages.feature.nlp_stages import OpLDA
    return OpLDA(k=k, max_iter=max_iter, seed=seed, **kw).set_input(self).get_output()


# ------------------------------------------------------------------------- round-3 DSL completions
@register(T.OPVector, "idf")
def _idf(self, min_doc_freq: int = 0):
    """``RichVectorFeature.idf`` (RichVectorFeature.scala:57)."""
    from ..stages.feature.text_stages import IDF
    return IDF(min_doc_freq=min_doc_freq).set_input(self).get_output()


@register(T.OPVector, "random_forest")
def _random_forest(self, label, max_depth: int = 5, max_bins: int = 32, min_instance_per_node: int = 1,
                   min_info_gain: float = 0.0, sub_sampling_rate: float = 1.0, num_trees: int = 20,
                   impurity: str = "entropy", seed: Optional[int] = None, thresholds=()):
    """``RichVectorFeature.randomForest`` (RichVectorFeature.scala:78-100): an OpRandomForestClassifier on
    (label, this vector)."""
    import random
    from ..models.trees import OpRandomForestClassifier
    params = dict(max_depth=max_depth, max_bins=max_bins, min_instances_per_node=min_instance_per_node,
                  min_info_gain=min_info_gain, subsampling_rate=sub_sampling_rate, num_trees=num_trees,
                  impurity=str(impurity).lower(), seed=random.getrandbits(31) if seed is None else int(seed))
    if thresholds:
        params["thresholds"] = list(thresholds)
    return OpRandomForestClassifier(**params).set_input(label, self).get_output()


@register((T.RealNN, T.Real, T.Integral), "deindexed")
def _deindexed(self, labels=(), unseen_name: str = "UnseenIndex", handle_invalid: str = "NoFilter"):
    """``RichNumericFeature.deindexed`` (RichNumericFeature.scala:418-432): index -> label, labels from the
    argument or from the string indexer that produced this feature."""
    from ..stages.feature.indexers import OpIndexToString, OpIndexToStringNoFilter
    if str(handle_invalid).lower() == "error":
        return OpIndexToString(labels=list(labels)).set_input(self).get_output()
    return OpIndexToStringNoFilter(labels=list(labels), unseen_name=unseen_name).set_input(self).get_output()


@register(T.Text, "to_multi_pick_list")
def _to_mpl(self):
    """``RichTextFeature.toMultiPickList`` (RichTextFeature.scala:53)."""
    from ..stages.feature.misc_stages import TextToMultiPickList
    return TextToMultiPickList().set_input(self).get_output()


@register(T.DateTime, "to_date_time_list")
def _to_dt_list(self):
    """``RichDateTimeFeature.toDateTimeList``."""
    from ..stages.feature.misc_stages import DateToListTransformer
    st = DateToListTransformer()
    st.output_type = T.DateTimeList
    return st.set_input(self).get_output()


@register(T.Date, "to_date_list")
def _to_date_list(self):
    """``RichDateFeature.toDateList`` (RichDateFeature.scala:55)."""
    from ..stages.feature.misc_stages import DateToListTransformer
    return DateToListTransformer().set_input(self).get_output()


@register(T.Phone, "is_valid_phone")
def _is_valid_phone(self, region_code, country_codes=None, is_strict: bool = False, default_region: str = "US"):
    """``RichTextFeature.isValidPhone(regionCode, ...)`` (RichTextFeature.scala:519-536): validity against
    the region given by a region-code / country-name feature."""
    from ..utils import phone as PH
    if country_codes is not None:
        PH.check_codes(country_codes)
    return TS.IsValidPhoneNumber(default_region=default_region, strict=is_strict,
                                 codes_and_countries=dict(country_codes) if country_codes else None) \
        .set_input(self, region_code).get_output()


@register(T.Phone, "parse_phone_with_region")
def _parse_phone_region(self, region_code, country_codes=None, is_strict: bool = False, default_region: str = "US"):
    """``RichTextFeature.parsePhone(regionCode, ...)``: E.164 form against the region feature."""
    return TS.ParsePhoneNumberWithRegion(default_region=default_region, strict=is_strict,
                                         codes_and_countries=dict(country_codes) if country_codes else None) \
        .set_input(self, region_code).get_output()


@register(T.Text, "to_ngram_similarity")
def _ngram_text_alias(self, other, n_gram_size: int = 3, to_lowercase: bool = True):
    return _ngram_text(self, other, n_gram_size, to_lowercase)


@register(T.MultiPickList, "to_ngram_similarity")
def _ngram_set_alias(self, other, n_gram_size: int = 3, to_lowercase: bool = True):
    return _ngram_set(self, other, n_gram_size, to_lowercase)

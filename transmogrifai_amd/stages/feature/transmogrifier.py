"""Automatic type-driven feature engineering: ``transmogrify``.

Reference: ``Transmogrifier.transmogrify`` (``core/.../impl/feature/Transmogrifier.scala:92-364``) and the
defaults ``TransmogrifierDefaults`` (``:52-88``); dispatch table in SURVEY.md Appendix B. Features are
grouped by exact type (sorted by type name for deterministic DAGs), each group gets its default
vectorizer, and all resulting vectors are concatenated by a ``VectorsCombiner``.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Sequence

from ...features import types as T
from ...features.feature import FeatureLike


class TransmogrifierDefaults:
    NullString = "NullIndicatorValue"
    OtherString = "OTHER"
    DefaultNumOfFeatures = 512
    MaxNumOfFeatures = 1 << 17
    DateListDefault = "SinceLast"
    ReferenceDate = None          # resolved to "now" when the stage first runs
    TopK = 20
    MinSupport = 10
    FillValue = 0
    BinaryFillValue = False
    HashWithIndex = False
    PrependFeatureName = True
    HashSpaceStrategy = "auto"
    CleanText = True
    CleanKeys = False
    BinaryFreq = False
    FillWithMode = True
    FillWithMean = True
    TrackNulls = True
    TrackInvalid = False
    TrackTextLen = False
    MinDocFrequency = 0
    MaxPercentCardinality = 1.0
    MinInfoGain = 0.01
    MaxCategoricalCardinality = 30
    CircularDateRepresentations = ("HourOfDay", "DayOfWeek", "DayOfMonth", "DayOfYear")
    DefaultRegion = "US"
    MinTokenLength = 1
    ToLowercase = True


_PIVOT_TYPES = (T.PickList, T.ComboBox, T.ID, T.Country, T.State, T.City, T.PostalCode, T.Street, T.Base64,
                T.URL, T.Email)


def _vectorize_group(t, feats: List[FeatureLike], label, D) -> List[FeatureLike]:
    from .text_stages import TextMapTransformer, PhoneValidator, OpHashingTF, IDF
    from .vectorizers import (BinaryVectorizer, DateListVectorizer, DateToUnitCircleTransformer,
                              GeolocationVectorizer, IntegralVectorizer, OpSetVectorizer, OpTextPivotVectorizer,
                              RealNNVectorizer, RealVectorizer, SmartTextVectorizer, VectorsCombiner)
    from .maps import map_vectorize

    def pivot(fs):
        return OpTextPivotVectorizer(top_k=D.TopK, min_support=D.MinSupport, clean_text=D.CleanText,
                                     track_nulls=D.TrackNulls,
                                     max_pct_cardinality=D.MaxPercentCardinality).set_input(fs).get_output()

    if t is T.OPVector:
        return list(feats)
    if t is T.RealNN:
        return [RealNNVectorizer().set_input(feats).get_output()]
    if t in (T.Real, T.Currency, T.Percent):
        st = RealVectorizer(track_nulls=D.TrackNulls, fill_value=float(D.FillValue))
        if D.FillWithMean:
            st.set_fill_with_mean()
        out = [st.set_input(feats).get_output()]
        if label is not None:
            from .bucketizers import DecisionTreeNumericBucketizer
            # RichRealFeature / RichIntegralFeature.vectorize with a label (RichNumericFeature.scala:329-336,
            # :660-667): autoBucketize(label, trackNulls = false, trackInvalid, minInfoGain)
            out += [DecisionTreeNumericBucketizer(track_nulls=False, track_invalid=getattr(D, "TrackInvalid", False),
                                                  min_info_gain=D.MinInfoGain)
                    .set_input(label, f).get_output() for f in feats]
        return out
    if t is T.Integral:
        st = IntegralVectorizer(track_nulls=D.TrackNulls, fill_value=float(D.FillValue))
        if D.FillWithMode:
            st.set_fill_with_mode()
        out = [st.set_input(feats).get_output()]
        if label is not None:
            from .bucketizers import DecisionTreeNumericBucketizer
            # RichRealFeature / RichIntegralFeature.vectorize with a label (RichNumericFeature.scala:329-336,
            # :660-667): autoBucketize(label, trackNulls = false, trackInvalid, minInfoGain)
            out += [DecisionTreeNumericBucketizer(track_nulls=False, track_invalid=getattr(D, "TrackInvalid", False),
                                                  min_info_gain=D.MinInfoGain)
                    .set_input(label, f).get_output() for f in feats]
        return out
    if t is T.Binary:
        return [BinaryVectorizer(fill_value=D.BinaryFillValue, track_nulls=D.TrackNulls).set_input(feats).get_output()]
    if t in (T.Date, T.DateTime):
        circ = [DateToUnitCircleTransformer(time_period=p).set_input(feats).get_output()
                for p in D.CircularDateRepresentations]
        since = DateListVectorizer(pivot=D.DateListDefault, reference_date=D.ReferenceDate,
                                   track_nulls=D.TrackNulls).set_input(feats).get_output()
        if not circ:
            return [since]
        return [VectorsCombiner().set_input(circ + [since]).get_output()]
    if t in (T.DateList, T.DateTimeList):
        return [DateListVectorizer(pivot=D.DateListDefault, reference_date=D.ReferenceDate,
                                   track_nulls=D.TrackNulls).set_input(feats).get_output()]
    if t is T.TextList:
        vecs = [IDF(min_doc_freq=D.MinDocFrequency).set_input(
            OpHashingTF(num_features=D.DefaultNumOfFeatures, binary=D.BinaryFreq).set_input(f).get_output()
        ).get_output() for f in feats]
        return [VectorsCombiner().set_input(vecs).get_output()] if len(vecs) > 1 else vecs
    if t is T.Geolocation:
        return [GeolocationVectorizer(track_nulls=D.TrackNulls).set_input(feats).get_output()]
    if t is T.MultiPickList:
        return [OpSetVectorizer(top_k=D.TopK, min_support=D.MinSupport, clean_text=D.CleanText,
                                track_nulls=D.TrackNulls).set_input(feats).get_output()]
    if t is T.Email:
        doms = [TextMapTransformer("EmailDomainToPickList", T.PickList).set_input(f).get_output() for f in feats]
        return [pivot(doms)]
    if t is T.URL:
        doms = [TextMapTransformer("URLDomainToPickList", T.PickList).set_input(f).get_output() for f in feats]
        return [pivot(doms)]
    if t is T.Base64:
        mts = [TextMapTransformer("MimeTypeDetector", T.PickList).set_input(f).get_output() for f in feats]
        return [pivot(mts)]
    if t is T.Phone:
        valid = [PhoneValidator(default_region=D.DefaultRegion).set_input(f).get_output() for f in feats]
        return [BinaryVectorizer(fill_value=D.BinaryFillValue, track_nulls=D.TrackNulls).set_input(valid).get_output()]
    if t in _PIVOT_TYPES:
        return [pivot(feats)]
    if t in (T.Text, T.TextArea):
        return [SmartTextVectorizer(max_cardinality=D.MaxCategoricalCardinality, track_nulls=D.TrackNulls,
                                    num_features=D.DefaultNumOfFeatures, hash_space_strategy=D.HashSpaceStrategy,
                                    min_token_length=D.MinTokenLength, to_lowercase=D.ToLowercase,
                                    prepend_feature_name=D.PrependFeatureName).set_input(feats).get_output()]
    if issubclass(t, T.OPMap):
        return map_vectorize(t, feats, label, D)
    raise ValueError(f"No vectorizer available for type {t.__name__}")


def transmogrify(features: Sequence[FeatureLike], label: Optional[FeatureLike] = None,
                 defaults=TransmogrifierDefaults) -> List[FeatureLike]:
    """Vectorize features by type; returns one vector feature per type group."""
    groups: "OrderedDict[type, List[FeatureLike]]" = OrderedDict()
    for f in features:
        groups.setdefault(f.wtype, []).append(f)
    out = []
    for t in sorted(groups, key=lambda t: t.type_name()):
        out.extend(_vectorize_group(t, groups[t], label, defaults))
    return out


def transmogrify_combined(features: Sequence[FeatureLike], label: Optional[FeatureLike] = None,
                          defaults=TransmogrifierDefaults) -> FeatureLike:
    """``Seq(features).transmogrify(label)`` = transmogrify + ``VectorsCombiner`` (``RichFeaturesCollection.scala:69-70``)."""
    from .vectorizers import VectorsCombiner
    vecs = transmogrify(features, label, defaults)
    return VectorsCombiner().set_input(vecs).get_output()

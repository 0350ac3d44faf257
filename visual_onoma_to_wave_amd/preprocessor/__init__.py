from .features import FeatureExtractor, normalize_features  # noqa: F401

"""transmogrifai_amd -- an MI355X-native AutoML engine for structured data."""
__version__ = "0.1.0"

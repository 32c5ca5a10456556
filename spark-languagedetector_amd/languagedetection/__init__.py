"""languagedetection -- MI355X-native drop-in for spark-languagedetector's hot path.

Mirrors org.apache.spark.ml.feature.languagedetection (LanguageDetector,
LanguageDetectorModel) over pandas DataFrames; the FIT counting and SCORE
kernels run on gfx950 through libldgpu.so (include/ldgpu.h).
"""
from .api import (FitValidationError, LanguageDetector, LanguageDetectorModel, LanguageDetectorModelReader,
                  LanguageDetectorModelWriter, NullPointerException, save_grams)
from .language import Language
from .preprocessing import LowerCasePreprocessor, PatternSyntaxException, SpecialCharPreprocessor
from .runtime import DeviceCounts, DeviceModel

__all__ = ["LanguageDetector", "LanguageDetectorModel", "LanguageDetectorModelReader", "LanguageDetectorModelWriter",
           "FitValidationError", "NullPointerException", "DeviceCounts", "DeviceModel", "save_grams",
           "LowerCasePreprocessor", "SpecialCharPreprocessor", "PatternSyntaxException", "Language"]

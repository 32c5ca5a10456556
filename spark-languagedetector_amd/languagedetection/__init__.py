"""languagedetection -- MI355X-native drop-in for spark-languagedetector's hot path.

Mirrors org.apache.spark.ml.feature.languagedetection (LanguageDetector,
LanguageDetectorModel) over pandas DataFrames; the FIT counting and SCORE
kernels run on gfx950 through libldgpu.so (include/ldgpu.h).
"""
from .api import (FitValidationError, FrozenTable, LanguageDetector, LanguageDetectorModel, LanguageDetectorModelReader,
                  LanguageDetectorModelWriter, NullPointerException, freeze_table, save_grams)
from .language import Language
from .preprocessing import LowerCasePreprocessor, PatternSyntaxException, SpecialCharPreprocessor
from .runtime import DeviceCounts, DeviceModel

__all__ = ["LanguageDetector", "LanguageDetectorModel", "LanguageDetectorModelReader", "LanguageDetectorModelWriter",
           "FitValidationError", "NullPointerException", "FrozenTable", "freeze_table", "DeviceCounts", "DeviceModel", "save_grams",
           "LowerCasePreprocessor", "SpecialCharPreprocessor", "PatternSyntaxException", "Language"]

"""Host-language mirror of pkg/fanal/analyzer/secret (undistro/trivy @ 2024-12-20)
and of the analyzer group's per-file fan-out for it, batched into arenas for the
MI355X engine (include/tsg_analyzer.h)."""
from .secret import (AnalysisInput, AnalysisResult, AnalyzerOptions, Collector, ExtractPrintableBytes,
                     FileInfo, IsBinary, NewSecretAnalyzer, SecretAnalyzer, SecretScannerOption, StripCR,
                     TypeSecret)

__all__ = ["AnalysisInput", "AnalysisResult", "AnalyzerOptions", "Collector", "ExtractPrintableBytes",
           "FileInfo", "IsBinary", "NewSecretAnalyzer", "SecretAnalyzer", "SecretScannerOption", "StripCR",
           "TypeSecret"]

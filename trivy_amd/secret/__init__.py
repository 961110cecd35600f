"""Host-language mirror of pkg/fanal/secret (undistro/trivy @ 2024-12-20).

Same names, argument meaning and error behaviour as the Go package, backed by
the MI355X engine in ``libtsg.so`` (include/tsg_scanner.h):

* ``ParseConfig(path)``   -- scanner.go:277-307 (YAML -> Config, severity normalised)
* ``NewScanner(config)``  -- scanner.go:320-364 (builtin + custom rules, enable/disable lists)
* ``Scanner.Scan(args)``  -- scanner.go:377-463, one file; ``Scanner.ScanBatch`` is the
  batched form the analyzer uses (arena + offsets, one GPU submission)
* ``Global.AllowPath``    -- scanner.go:57-59

There is no CPU fallback: constructing a Scanner without a HIP device raises.
"""
from .config import (AllowRule, Config, ExcludeBlock, Rule, ParseConfig, convert_severity,
                     builtin_rules, builtin_allow_rules)
from .scanner import (ScanArgs, Scanner, NewScanner, Secret, SecretFinding, Code, Line, HostRegister)

__all__ = ["AllowRule", "Config", "ExcludeBlock", "Rule", "ParseConfig", "convert_severity",
           "builtin_rules", "builtin_allow_rules", "ScanArgs", "Scanner", "NewScanner", "Secret",
           "SecretFinding", "Code", "Line", "HostRegister"]

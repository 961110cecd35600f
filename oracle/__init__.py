"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the secret-scanning hot path.

Nothing under ``trivy_amd/`` imports this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker / the reported CPU baseline -- never as the thing measured
or shipped.

What it is: a restatement, in Python, of the reference's CPU algorithm for
``pkg/fanal/secret.Scanner.Scan`` (undistro/trivy @ 2024-12-20,
``pkg/fanal/secret/scanner.go:102-558``) on top of a restatement of the Go
standard-library pieces it relies on (go1.22.9, ``go.mod:3``):

* ``regexp`` / ``regexp/syntax``  -> ``oracle.goregexp``: a Go-syntax parser whose
  output is re-emitted as an explicit CPython ``re`` pattern (leftmost-first
  backtracking == Go's leftmost-first semantics for this syntax), with Go's
  UTF-8 rune model (invalid byte -> U+FFFD, width 1) mapped onto
  ``surrogateescape`` code points;
* ``bytes.ToLower`` / ``unicode.ToLower`` / ``strconv.Quote`` -> ``oracle.gostd``;
* ``sort.Slice`` (pdqsort)       -> ``oracle.gosort``.

Parity pinning: every case of ``pkg/fanal/secret/scanner_test.go:22-1351`` and
``integration/testdata/secrets.json.golden`` (transcribed to
``tests/golden/``) must pass -- ``tests/test_oracle_golden.py``.  Behaviour those
fixtures do not exercise (non-ASCII case folding, invalid UTF-8, pdqsort tie
order above 12 findings) is a restatement and is marked "parity unpinned" in
DESIGN.md.  The Go toolchain is absent from the image, so the reference itself
cannot be run.
"""

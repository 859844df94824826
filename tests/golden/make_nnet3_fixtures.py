"""Extracts the nnet3 text fixtures held by the reference's own tests
(internal/nnet/weight_loader_test.go: the Go raw-string inputs of TestParseNnet3Text,
TestParseRealBatchNormLine, TestParseInlineVector, TestParseRealPrefinalLine) into
tests/golden/nnet3_*.txt. Run once in the build container (the reference is not on the
GPU box); the outputs are data — real `nnet3-copy --binary=false` text snippets."""
import os
import re
import sys

SRC = "/root/reference/internal/nnet/weight_loader_test.go"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    src = open(SRC).read()
    raws = re.findall(r"`([^`]*)`", src)
    names = ["components", "bn_line", "inline_vector", "prefinal_line"]
    assert len(raws) == len(names), len(raws)
    for n, r in zip(names, raws):
        with open(os.path.join(OUT, f"nnet3_{n}.txt"), "w") as f:
            f.write(r)
        print(n, len(r), "bytes")


if __name__ == "__main__":
    sys.exit(main())

#!/bin/sh
# Regenerates reference_exports.txt: the dynamic symbol table (defined text symbols)
# of the reference's shipped libraries, read with nm (the binaries are never loaded
# or run). Run in the build container, where /root/reference exists.
set -e
R=/root/reference/cpp/build
OUT=$(dirname "$0")/reference_exports.txt
: > "$OUT"
for lib in libkaldi_fp16.so libkaldi_fp16_cgo.so libkaldi_fp16_den.so; do
    nm -D --defined-only "$R/$lib" | awk -v L="$lib" '$2=="T" && $3 !~ /^_/ {print L, $3}' | sort >> "$OUT"
done

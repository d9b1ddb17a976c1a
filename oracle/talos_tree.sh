#!/bin/bash
# talos_tree.sh — TEST INFRASTRUCTURE ONLY.
#
# Prepares the TaLoS-patched LibreSSL tree (BASELINE configs[0]: the
# Makefile.nosgx build) in a scratch directory OUTSIDE the repository:
# /root/reference stays read-only and nothing of it is copied into the repo.
# The tree is the reference's own src/libressl-2.4.1 with its own
# src/talos/patch_libressl.sh applied (that script copies src/talos/enclaveshim/*
# into crypto/ and applies src/talos/patch/*.patch with patch -p0), exactly as
# SURVEY.md §8c did.  oracle/Makefile (target `talos`) then compiles it.
#
# usage: talos_tree.sh DEST   (default /tmp/talos_ref); no-op when DEST is ready
set -euo pipefail
REFSRC=${REFSRC:-/root/reference/src}
DEST=${1:-/tmp/talos_ref}
[ -f "$DEST/.patched" ] && exit 0
[ -d "$REFSRC/talos" ] || { echo "no reference tree at $REFSRC" >&2; exit 1; }
rm -rf "$DEST"
mkdir -p "$DEST"
cp -r "$REFSRC/libressl-2.4.1" "$REFSRC/talos" "$DEST/"
chmod -R u+w "$DEST"
(cd "$DEST/talos" && bash ./patch_libressl.sh > "$DEST/patch.log" 2>&1)
if grep -qi "rej\|FAILED" "$DEST/patch.log"; then
  echo "patch_libressl.sh reported rejects (see $DEST/patch.log)" >&2
  exit 1
fi
touch "$DEST/.patched"

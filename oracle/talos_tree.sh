#!/bin/bash
# talos_tree.sh — TEST INFRASTRUCTURE ONLY.
#
# Prepares the TaLoS-patched LibreSSL tree (BASELINE configs[0]: the
# Makefile.nosgx build) in a scratch directory OUTSIDE the repository:
# /root/reference stays read-only and nothing of it is copied into the repo.
# The tree is the reference's own src/libressl-2.4.1 with the TaLoS changes
# applied the way src/talos/patch_libressl.sh describes them: the files of
# src/talos/enclaveshim/ copied into crypto/, then every src/talos/patch/*.patch
# applied with patch -p0 from the libressl directory.  Those two steps are done
# here; no script from the reference tree is ever executed.
# oracle/Makefile (target `talos`) then compiles the tree.
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
cp "$DEST"/talos/enclaveshim/* "$DEST/libressl-2.4.1/crypto/"
: > "$DEST/patch.log"
for p in "$DEST"/talos/patch/*.patch; do
  (cd "$DEST/libressl-2.4.1" && patch -p0 --batch -i "$p") >> "$DEST/patch.log" 2>&1 || {
    echo "patch $p failed (see $DEST/patch.log)" >&2
    exit 1
  }
done
if grep -qi "rej\|FAILED" "$DEST/patch.log"; then
  echo "the TaLoS patches reported rejects (see $DEST/patch.log)" >&2
  exit 1
fi
touch "$DEST/.patched"

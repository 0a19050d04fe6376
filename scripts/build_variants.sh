#!/bin/bash
# Build kernel variants (compile-time knobs) into abvar/<name>/libraingun_hip.so
# usage: scripts/build_variants.sh name1="-DKNOB=1 ..." name2="..."
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name="${spec%%=*}"; flags="${spec#*=}"
  mkdir -p abvar/$name
  make -s -B -C raingun_amd/csrc OUT=$PWD/abvar/$name/libraingun_hip.so EXTRA="$flags" >/dev/null
  echo "$flags" > abvar/$name/flags.txt
  echo "built $name: $flags"
done

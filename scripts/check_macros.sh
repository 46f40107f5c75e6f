#!/bin/bash
# usage: scripts/check_macros.sh <source.hip> [-DNAME[=v] ...]
# Fails if a -D macro is not referenced by the source or the headers of
# ogbench_amd/csrc (a variant built with a removed macro would silently be
# the default kernel).  Other flags pass through unchecked.
set -eu
src=$1; shift
dir=$(dirname "$src")
for a in "$@"; do
  case "$a" in
    -D*)
      m=${a#-D}; m=${m%%=*}
      if ! grep -qw -- "$m" "$src" "$dir"/*.h ; then
        echo "unknown macro $m: not referenced by $src or $dir/*.h" >&2
        exit 2
      fi ;;
  esac
done

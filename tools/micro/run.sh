#!/bin/bash
# run every tools/micro binary given on the command line (1024 waves, then one wave), each under its own limit
cd "$(dirname "$0")" || exit 1
for b in "$@"; do
  echo "== $b"
  timeout -k 5 60 ./$b 1024 20 || exit 1
  timeout -k 5 60 ./$b 1 20 || exit 1
done

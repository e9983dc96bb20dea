#!/bin/bash
# every input of work/ood through tools/decode_file: status, re-plans and the
# error key of the first failing frame (classifies what stays out of domain)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in ${1:-work/ood}/*.zst; do
  fl=0; case $f in *_p1.zst) fl=1;; esac
  echo "== $f $(timeout -k 10 60 tools/decode_file "$f" $fl | tail -1)" || exit 1
done

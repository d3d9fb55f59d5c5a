#!/bin/bash
# Build libmq_aead.so of git revision $1 into milli_quic_amd/csrc/build/rev_$1.so (A/B timing
# against the working tree with tools/ab.py). Diagnostic only.
set -e
REV=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/include $T/milli_quic_amd/csrc
git -C $ROOT show $REV:include/mq_aead.h > $T/include/mq_aead.h
for f in $(git -C $ROOT ls-tree --name-only $REV milli_quic_amd/csrc/); do
  git -C $ROOT show $REV:$f > $T/$f
done
make -C $T/milli_quic_amd/csrc -s -j8 >/dev/null
mkdir -p $ROOT/milli_quic_amd/csrc/build
cp $T/milli_quic_amd/libmq_aead.so $ROOT/milli_quic_amd/csrc/build/rev_$REV.so
rm -rf $T
echo $ROOT/milli_quic_amd/csrc/build/rev_$REV.so

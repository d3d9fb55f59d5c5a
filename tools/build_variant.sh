#!/bin/bash
# Build a variant of libmq_aead.so whose mq_chacha.hip / mq_aes.hip are compiled with extra
# flags (e.g. -DMQ_CC_SEAL_WAVES=8) into tools/ab_libs/NAME.so, for A/B timing with tools/ab.py.
# The other objects come from the product build (make first). Diagnostic only.
# Usage: tools/build_variant.sh NAME "FLAGS" [SRC...]   (SRC default: mq_chacha.hip)
set -e
NAME=$1; FLAGS=$2; shift 2
SRCS=${@:-mq_chacha.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/milli_quic_amd/csrc
O=$C/build/var_$NAME
mkdir -p $O $ROOT/tools/ab_libs
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-align-mismatch"
OBJS=""
for f in mq_chacha.hip mq_aes.hip mq_partition.hip mq_record.hip mq_derive.hip mq_send.hip mq_recv.hip mq_resident.hip mq_host.cpp; do
  if [[ " $SRCS " == *" $f "* ]]; then
    /opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c $C/$f -o $O/$f.o
    OBJS="$OBJS $O/$f.o"
  else
    OBJS="$OBJS $C/build/$f.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/ab_libs/$NAME.so $OBJS
echo $ROOT/tools/ab_libs/$NAME.so

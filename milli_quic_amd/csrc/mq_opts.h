// mq_opts.h — diagnostic switches of libmq_aead.so (A/B builds, tests that run two paths of one
// batch). None of them changes a result, only which kernels compute it.
//
// Each switch is an atomic word, filled ONCE from its MQ_* environment variable the first time any
// switch is read, and settable at run time with mq_debug_option (include/mq_aead.h). Hot paths
// read the word (one relaxed load), never the environment: getenv on every call raced with setenv
// in other threads and let a switch change between the walks of one receive batch.
#ifndef MQ_OPTS_H
#define MQ_OPTS_H

namespace mq {

enum class Opt : int {
  CcNarrow,           // MQ_CC_NARROW: 0 / 1 forces the wide / narrow flat ChaCha20 kernels; 0 also
                      // turns the partition's narrow regions off
  CcLong,             // MQ_CC_LONG: 0 / 1 / 2 forces the 10-, 13- or 20-KiB flat ChaCha20 images
  CcList,             // MQ_CC_LIST: 0 / 1 forces the one-shot / persistent ChaCha20 list grids
  HpFork,             // MQ_HP_FORK: 0 runs the mixed open pre-pass after the partition on the caller's stream
  AesSeg,             // MQ_AES_SEG: 0 never / 1 always runs the key-segmented AES kernels when keyed
  ProtectFused,       // MQ_PROTECT_FUSED: 0 keeps the two-kernel ChaCha20 protect composite
  Resident,           // MQ_RESIDENT: 0 sends per-packet calls through a launch instead of the resident kernel
  ResidentTimeoutUs,  // MQ_RESIDENT_TIMEOUT_US: how long a per-packet call waits for the resident kernel
  RecvSeg,            // MQ_RECV_SEG: receive-walk segment length (0 = one segment per run)
  AesHotSeg,          // MQ_AES_HOT_SEG: 0 runs a partition's hot AES segment on the tile kernel, not the slice kernel
  AesNarrow,          // MQ_AES_NARROW: 0 / 1 / 2 forces 8 / 4 / 2 lanes per packet in the single-key AES kernels
  Count
};

// The switch's value, or -1 when it is unset (the product behaviour).
long opt(Opt o);

}  // namespace mq

#endif

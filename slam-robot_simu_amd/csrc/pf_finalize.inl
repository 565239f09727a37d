// pf_finalize.inl -- layout constants of the one-workgroup reductions over the
// fused blocks' partials, shared by the sharded step's record (pf_dist.inl:
// dist_reduce_kernel).  The single-GPU step end is pf_stepend.inl.

constexpr int kFinThreads = 512;
constexpr int kFinWaves = kFinThreads / 64;
constexpr int kFinRegBlocks = 2048 / kFinThreads;   // fused blocks held in registers per lane (2048)
constexpr int kFinLeafLanes = 4;            // lanes per 8192-element buffer (16 leaves each)
constexpr int kFinBufPerRound = kFinThreads / kFinLeafLanes;   // 128 buffers per round

// A lane of the np.sum pass takes 4 consecutive fused blocks of a buffer: each
// block left the pairwise sum of its four 128-element leaves (a perfect
// subtree of the buffer's tree), so (b0 + b1) + (b2 + b3) is the lane's
// 16-leaf subtree.
static_assert(kSumChunk == 16 * kPartPer, "a buffer is 16 fused blocks, 4 per np.sum lane");

// register block k of lane t (k < kFinRegBlocks): neighbour pairs, increasing in k
__device__ __forceinline__ int64_t fin_blk(const int t, const int k) {
    static_assert(kFinRegBlocks % 2 == 0, "pairs of blocks");
    return 2 * (int64_t)t + (k & 1) + 2 * (int64_t)kFinThreads * (k >> 1);
}

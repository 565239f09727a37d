// pf_shard_api.inl -- C-ABI of the sharded particle filter (included by pf_api.hip).
//
// One handle per GPU holds particles [gbase, gbase + n_local) of a filter of
// n_global particles.  The caller runs the phases below in order and moves
// the small exchange buffers between ranks (slamhip/shard.py does it with
// torch.distributed, i.e. RCCL over xGMI on MI355X).  All exchange buffers are
// device pointers owned by the caller; everything runs on the handle's stream
// (slam_pf_set_stream lets it be the caller's stream).

namespace {

int shard_ensure(slam_pf* h, int32_t world) {
    ShardScratch& s = h->sh;
    if (s.world == world && s.meta_dev) return SLAM_OK;
    int rc;
    if ((rc = dalloc(h, &s.meta_dev, 2 * (size_t)world)) || (rc = dalloc(h, &s.gb_dev, world + 1)) ||
        (rc = dalloc(h, &s.cnt_dev, 2 * (size_t)world)) || (rc = dalloc(h, &s.off_dev, world + 1)) ||
        (rc = dalloc(h, &s.spec_base, 1)) || (rc = dalloc(h, &s.k_base, 1)) ||
        (rc = dalloc(h, &s.nspec_g, 1)) || (rc = dalloc(h, &s.ktot_g, 1)) ||
        (rc = dalloc(h, &s.base_off, 1)) || (rc = dalloc(h, &s.c_left, 1)) ||
        (rc = dalloc(h, &s.hi, (size_t)h->n)))
        return rc;
    s.world = world;
    return SLAM_OK;
}

}  // namespace

extern "C" {

int slam_pf_shard_sizes(slam_pf* h, int64_t* out) {
    SLAM_ARG_CHECK(h && out, "slam_pf_shard_sizes: NULL argument");
    out[0] = h->nchunks;
    out[1] = (int64_t)sizeof(ShardRecord);
    out[2] = (int64_t)sizeof(SpecialIn);
    out[3] = (int64_t)sizeof(ShardItem);
    return SLAM_OK;
}

int slam_pf_shard_begin(slam_pf* h, const double* control, const double* z, const double* noise,
                        double u_resample, int32_t resample) {
    SLAM_ARG_CHECK(h && control && (z || h->nl == 0), "slam_pf_shard_begin: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc;
    if ((rc = stage_inputs(h, control, z, noise, u_resample))) return rc;
    h->sh.host_noise = noise != nullptr;
    h->resample_next = resample ? 1 : 0;
    return set_flag(h, kFlagResample, 0);
}

int slam_pf_shard_scan_local(slam_pf* h, double* d_total) {
    SLAM_ARG_CHECK(h && d_total, "slam_pf_shard_scan_local: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = launch_bsum(h);
    if (rc) return rc;
    SLAM_HIP_TRY(hipMemcpyAsync(d_total, h->boff + h->nb_norm, 8, hipMemcpyDeviceToDevice, h->stream));
    return SLAM_OK;
}

int slam_pf_shard_classify(slam_pf* h, const double* d_totals, int32_t rank, int32_t world,
                           int64_t* d_meta) {
    SLAM_ARG_CHECK(h && d_totals && d_meta && rank >= 0 && rank < world, "slam_pf_shard_classify: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = shard_ensure(h, world);
    if (rc) return rc;
    hipStream_t s = h->stream;
    const int nb = h->nb_scan;
    const double delta = 4.0 * (double)h->n_global * 0x1p-53 + 0x1p-45;
    shard_prefix_kernel<<<1, 64, 0, s>>>(d_totals, rank, h->sh.base_off);
    scan_classify_kernel<<<nb, kScanThreads, 0, s>>>(
        h->w, h->n, h->boff, h->sh.base_off, h->c, h->kincl, h->fexcl, h->bk, h->bf, h->boffk,
        h->bofff, h->ktot, h->nspec, delta, h->gbase, h->tk + 2 * kTicketWords, h->flags, 1,
        nullptr, h->pc.np_recip, kNormPer);
    scan_emit_kernel<<<nb, kScanThreads, 0, s>>>(h->w, h->n, h->c, h->kincl, h->fexcl, h->boffk,
                                                 h->bofff, h->spec_in, h->gbase, h->spec_out,
                                                 h->nspec, h->ktot, 0, h->c, h->tk + 2 * kTicketWords,
                                                 h->flags, 1, nullptr, h->pc.np_recip);
    shard_meta_kernel<<<1, 64, 0, s>>>(h->nspec, h->ktot, d_meta);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int slam_pf_shard_export_specials(slam_pf* h, int64_t count, void* d_dst) {
    SLAM_ARG_CHECK(h && (d_dst || count == 0) && count >= 0 && count <= h->n,
                   "slam_pf_shard_export_specials: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    if (count)
        SLAM_HIP_TRY(hipMemcpyAsync(d_dst, h->spec_in, count * sizeof(SpecialIn),
                                    hipMemcpyDeviceToDevice, h->stream));
    return SLAM_OK;
}

// meta: HOST array world x (nspec, ktot) -- the gathered classify metadata
int slam_pf_shard_fold(slam_pf* h, const void* d_lists, int64_t cap, const int64_t* meta,
                       int32_t world, int32_t rank) {
    SLAM_ARG_CHECK(h && d_lists && meta && rank >= 0 && rank < world, "slam_pf_shard_fold: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = shard_ensure(h, world);
    if (rc) return rc;
    ShardScratch& S = h->sh;
    int64_t total = 0;
    uint64_t ktot = 0;
    int64_t nb = 0;
    uint64_t kb = 0;
    for (int r = 0; r < world; ++r) {
        if (r == rank) {
            nb = total;
            kb = ktot;
        }
        total += meta[2 * r];
        ktot += (uint64_t)meta[2 * r + 1];
    }
    SLAM_ARG_CHECK(total <= h->n_global, "slam_pf_shard_fold: inconsistent metadata");
    if (S.spec_cap < total) {
        for (void* p : {(void*)S.spec_g, (void*)S.spec_go})
            if (p) {
                (void)hipFree(p);
                h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), p), h->allocs.end());
            }
        if ((rc = dalloc(h, &S.spec_g, (size_t)total)) || (rc = dalloc(h, &S.spec_go, (size_t)total)))
            return rc;
        S.spec_cap = total;
    }
    hipStream_t s = h->stream;
    SLAM_HIP_TRY(hipMemcpyAsync(S.meta_dev, meta, 2 * world * sizeof(int64_t), hipMemcpyHostToDevice, s));
    const int32_t nb32 = (int32_t)nb, tot32 = (int32_t)total;
    SLAM_HIP_TRY(hipMemcpyAsync(S.spec_base, &nb32, 4, hipMemcpyHostToDevice, s));
    SLAM_HIP_TRY(hipMemcpyAsync(S.k_base, &kb, 8, hipMemcpyHostToDevice, s));
    SLAM_HIP_TRY(hipMemcpyAsync(S.nspec_g, &tot32, 4, hipMemcpyHostToDevice, s));
    SLAM_HIP_TRY(hipMemcpyAsync(S.ktot_g, &ktot, 8, hipMemcpyHostToDevice, s));
    int64_t maxc = 1;
    for (int r = 0; r < world; ++r) maxc = std::max<int64_t>(maxc, meta[2 * r]);
    dim3 grid((unsigned)std::min<int64_t>(256, (maxc + 255) / 256), (unsigned)world);
    shard_concat_kernel<<<grid, 256, 0, s>>>((const SpecialIn*)d_lists, cap, S.meta_dev, world, S.spec_g);
    scan_fold_kernel<<<1, 256, 0, s>>>(S.spec_g, S.spec_go, S.nspec_g, S.ktot_g, h->n_global,
                                       h->flags, h->w, h->c, 0);
    scan_expand_kernel<<<h->nb_scan, kScanThreads, 0, s>>>(h->n, h->kincl, h->fexcl, h->boffk,
                                                           h->bofff, S.spec_go, h->c, h->flags,
                                                           S.spec_base, S.k_base, 1);
    shard_left_kernel<<<1, 64, 0, s>>>(S.spec_go, S.spec_base, S.k_base, h->gbase, S.c_left);
    SLAM_HIP_TRY(hipGetLastError());
    // the fold's verification must hold across shards (no sequential fallback)
    int32_t fb = 0;
    SLAM_HIP_TRY(hipMemcpyAsync(&fb, h->flags + kFlagFallback, 4, hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    if (fb) return fail(SLAM_ERR_STATE, "sharded exact cumsum: run verification failed");
    return SLAM_OK;
}

// gb: HOST array of world+1 shard bases; send_counts: HOST out (world)
int slam_pf_shard_plan(slam_pf* h, const int64_t* gb, int32_t world, int64_t* send_counts) {
    SLAM_ARG_CHECK(h && gb && send_counts, "slam_pf_shard_plan: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = shard_ensure(h, world);
    if (rc) return rc;
    ShardScratch& S = h->sh;
    hipStream_t s = h->stream;
    S.gb.assign(gb, gb + world + 1);
    SLAM_HIP_TRY(hipMemcpyAsync(S.gb_dev, S.gb.data(), (world + 1) * 8, hipMemcpyHostToDevice, s));
    shard_hi_kernel<<<grid_for(h->n, 256), 256, 0, s>>>(h->c, h->n, h->gbase, h->n_global,
                                                       h->pc.rstep, h->ofs, h->pc.np_recip,
                                                       h->cfg.seed, h->ctr, S.hi, h->flags);
    int64_t* lo0_dev = S.off_dev + world;      // scratch word
    shard_dest_kernel<<<1, 64, 0, s>>>(S.hi, h->n, S.c_left, h->n_global, h->pc.rstep, h->ofs,
                                       h->pc.np_recip, h->cfg.seed, h->ctr, S.gb_dev, world,
                                       S.cnt_dev, lo0_dev);
    SLAM_HIP_TRY(hipGetLastError());
    std::vector<int64_t> se(2 * world);
    SLAM_HIP_TRY(hipMemcpyAsync(se.data(), S.cnt_dev, se.size() * 8, hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipMemcpyAsync(&S.lo0_host, lo0_dev, 8, hipMemcpyDeviceToHost, s));
    SLAM_HIP_TRY(hipStreamSynchronize(s));
    S.start.resize(world);
    S.end.resize(world);
    S.off.assign(world + 1, 0);
    for (int d = 0; d < world; ++d) {
        S.start[d] = se[2 * d];
        S.end[d] = se[2 * d + 1];
        send_counts[d] = S.end[d] - S.start[d];
        S.off[d + 1] = S.off[d] + send_counts[d];
    }
    S.n_send = S.off[world];
    return SLAM_OK;
}

int slam_pf_shard_export_items(slam_pf* h, void* d_send) {
    SLAM_ARG_CHECK(h && (d_send || h->sh.n_send == 0), "slam_pf_shard_export_items: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    ShardScratch& S = h->sh;
    if (S.n_send == 0) return SLAM_OK;
    hipStream_t s = h->stream;
    SLAM_HIP_TRY(hipMemcpyAsync(S.off_dev, S.off.data(), S.world * 8, hipMemcpyHostToDevice, s));
    const int c = h->cur;
    shard_pack_kernel<<<grid_for(S.n_send, 256), 256, 0, s>>>(
        h->x[c], h->y[c], h->th[c], S.hi, S.lo0_host, S.cnt_dev, S.off_dev, S.gb_dev, S.world,
        S.n_send, (ShardItem*)d_send);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipStreamSynchronize(s));     // d_send complete before the exchange
    return SLAM_OK;
}

int slam_pf_shard_import_items(slam_pf* h, const void* d_recv, int64_t n_items) {
    SLAM_ARG_CHECK(h && d_recv && n_items > 0, "slam_pf_shard_import_items: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    const int c = h->cur;
    shard_unpack_kernel<<<grid_for(h->n, 256), 256, 0, h->stream>>>(
        (const ShardItem*)d_recv, n_items, h->n, h->gbase, h->x[c], h->y[c], h->th[c], h->w,
        h->pc.np_recip, h->flags);
    SLAM_HIP_TRY(hipGetLastError());
    return set_flag(h, kFlagResample, 2);       // already gathered: the fused kernel uses w = 1/N
}

int slam_pf_shard_predict_update(slam_pf* h, double* d_partials) {
    SLAM_ARG_CHECK(h && d_partials, "slam_pf_shard_predict_update: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    int rc = launch_fused(h, h->cfg.motion, h->sh.host_noise);
    if (rc) return rc;
    chunk_sum_kernel<<<h->nchunks, 512, 0, h->stream>>>(h->w_un, h->n, h->part, h->tail_leaves,
                                                         h->tail_ops, h->n_tail_leaves,
                                                         h->n_tail_ops, h->tk, nullptr);
    SLAM_HIP_TRY(hipGetLastError());
    SLAM_HIP_TRY(hipMemcpyAsync(d_partials, h->part, h->nchunks * 8, hipMemcpyDeviceToDevice, h->stream));
    return SLAM_OK;
}

int slam_pf_shard_normalize(slam_pf* h, const double* d_all_partials, int64_t nparts, void* d_record) {
    SLAM_ARG_CHECK(h && d_all_partials && d_record && nparts > 0, "slam_pf_shard_normalize: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const int c = h->cur;
    shard_fold_sum_kernel<<<1, 256, 0, s>>>(d_all_partials, nparts, h->wsum);
    normalize_kernel<<<h->nb_norm, kNormThreads, 0, s>>>(h->n, h->w_un, h->w, h->wsum,
                                                          h->pc.np_recip, h->x[c], h->y[c],
                                                          h->th[c], h->refp, h->bp, h->bsum,
                                                          h->gbase);
    shard_record_kernel<<<1, kNormThreads, 0, s>>>(h->bp, h->nb_norm, h->x[c], h->y[c], h->th[c],
                                                   h->gbase, (ShardRecord*)d_record);
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int slam_pf_shard_finish(slam_pf* h, const void* d_all_records, int32_t world, slam_pf_result* res) {
    SLAM_ARG_CHECK(h && d_all_records && world > 0, "slam_pf_shard_finish: bad argument");
    SLAM_HIP_TRY(hipSetDevice(h->device));
    shard_finish_kernel<<<1, 64, 0, h->stream>>>((const ShardRecord*)d_all_records, world, h->refp,
                                                 h->wsum, h->flags, h->cfg.ess_threshold,
                                                 h->res_dev, h->resample_next);
    SLAM_HIP_TRY(hipGetLastError());
    h->stepno++;
    const int rc = sync_results(h, 0, 1, res);
    if (h->res_host[0].status & 4)
        return fail(SLAM_ERR_COMM, "sharded resample: received particles do not cover this shard");
    return rc;
}

}  // extern "C"

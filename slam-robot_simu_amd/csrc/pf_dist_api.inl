// pf_dist_api.inl -- C-ABI of the sharded particle filter's device-resident
// step (included by pf_api.hip; kernels in pf_dist.inl).
//
// A slam_dist groups the shards this process holds: all of them (LOCAL: tests,
// or several shards on one GPU -- one shared stream, kernels enqueued phase by
// phase across the shards) or one (one process per GPU).  Each held shard owns
// an exchange region in fine-grained device memory; in the one-per-process form
// the regions are exported with hipIpcGetMemHandle, gathered by the caller's
// bootstrap (slam_comm_all_gather_host over RCCL, or any other channel) and
// opened by every peer.

struct slam_dist {
    int world = 1, rank0 = 0, nloc = 1;
    bool local = false;
    int device = 0;
    std::vector<slam_pf*> sh;                 // held shards, rank order
    DistLayout L;
    std::vector<char*> xbuf;                  // exchange region of each held shard
    std::vector<DistPeers> peers;             // per held shard
    std::vector<DistScratch*> scr;
    std::vector<SpecialIn*> spec_g;
    std::vector<SpecialOut*> spec_go;
    std::vector<int64_t*> hi;
    std::vector<int32_t*> bsel, bsel_off;
    std::vector<unsigned*> tk;                // 4 ticket blocks per held shard
    std::vector<void*> dallocs;
    std::vector<void*> opened;                // IPC mappings of peer regions
    hipStream_t stream = nullptr;             // LOCAL: the shared stream
    bool connected = false;
    bool merged = false;                      // one-launch resample exchange (one held shard, co-resident grid)
    bool merged_ok = false;
    hipGraphExec_t graph[2] = {nullptr, nullptr};     // kGraphSteps steps per parity
    hipGraphExec_t graph1[2] = {nullptr, nullptr};    // one step per parity
    // collective mode (slam_dist_set_collective): host-orchestrated steps, the
    // exchanges as RCCL collectives (one held shard) or device copies between
    // the held shards' regions (LOCAL)
    bool coll = false;
    slam_comm* comm = nullptr;
    int64_t* cnt_mat = nullptr;               // [world][world] gathered item counts (device)
    int64_t* hst = nullptr;                   // pinned host: counts / headers
};

namespace {

int dist_alloc(slam_dist* d, void** p, size_t bytes) {
    SLAM_HIP_TRY(hipMalloc(p, bytes ? bytes : 8));
    d->dallocs.push_back(*p);
    return SLAM_OK;
}

void dist_drop_graphs(slam_dist* d) {
    for (auto* gs : {d->graph, d->graph1})
        for (int k = 0; k < 2; ++k)
            if (gs[k]) {
                (void)hipGraphExecDestroy(gs[k]);
                gs[k] = nullptr;
            }
}

// every phase of one step, phase-major across the held shards
int dist_enqueue_step(slam_dist* d) {
    const int m = d->nloc;
    if (d->merged) {                                      // the resample exchange in one launch
        slam_pf* h = d->sh[0];
        const double delta = 4.0 * (double)h->n_global * 0x1p-53 + 0x1p-45;
        const int c = h->cur;
        dist_resample_merged_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
            h->w_un, h->s_cur, h->pc.np_recip, h->n, h->boff, delta, h->stage, h->bk, h->bf,
            h->boffk, h->bofff, h->ktot, h->nspec, d->tk[0], h->flags, d->spec_go[0], d->scr[0],
            h->x[c], h->y[c], h->th[c], h->dp.mark,
            h->dp.carry, d->peers[0], step_io(h), h->pc, h->cfg.seed, h->nb_part);
    }
    for (int i = 0; i < m && !d->merged; ++i) {           // exact cumsum: classify
        slam_pf* h = d->sh[i];
        const double delta = 4.0 * (double)h->n_global * 0x1p-53 + 0x1p-45;
        scan_classify_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
            h->w_un, h->n, h->boff, &d->scr[i]->base_off, h->c, h->kincl, h->fexcl, h->bk, h->bf,
            h->boffk, h->bofff, h->ktot, h->nspec, delta, h->gbase, h->tk + 2 * kTicketWords,
            h->flags, 0, h->s_cur, h->pc.np_recip, kPartPer);
    }
    for (int i = 0; i < m && !d->merged; ++i) {           // emit + push specials
        slam_pf* h = d->sh[i];
        dist_emit_push_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
            h->w_un, h->s_cur, h->pc.np_recip, h->n, h->c, h->kincl, h->fexcl, h->boffk, h->bofff,
            h->spec_in, h->gbase, h->nspec, h->ktot, d->tk[i], h->flags, d->peers[i], step_io(h));
    }
    for (int i = 0; i < m && !d->merged; ++i) {           // fold (waits for the specials)
        slam_pf* h = d->sh[i];
        dist_fold_kernel<<<1, 256, 0, h->stream>>>(d->spec_g[i], d->spec_go[i], h->n_global,
                                                   h->flags, d->scr[i], d->peers[i], step_io(h),
                                                   h->pc.rstep, h->pc.np_recip, h->cfg.seed);
    }
    for (int i = 0; i < m && !d->merged; ++i) {           // expand + hi + counts
        slam_pf* h = d->sh[i];
        dist_expand_hi_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
            h->n, h->kincl, h->fexcl, h->boffk, h->bofff, d->spec_go[i], h->c, d->hi[i], d->bsel[i],
            d->bsel_off[i], d->tk[i] + kTicketWords, h->flags, d->scr[i], d->peers[i], step_io(h),
            h->n_global, h->pc.rstep, h->pc.np_recip, h->cfg.seed);
    }
    for (int i = 0; i < m && !d->merged; ++i) {           // pack + push items
        slam_pf* h = d->sh[i];
        const int c = h->cur;
        dist_pack_push_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
            h->n, h->x[c], h->y[c], h->th[c], d->hi[i], d->bsel_off[i], d->tk[i] + 2 * kTicketWords,
            h->flags, d->scr[i], d->peers[i], step_io(h));
    }
    for (int i = 0; i < m && !d->merged; ++i) {           // unpack (waits for the items)
        slam_pf* h = d->sh[i];
        const int c = h->cur;
        dist_unpack_kernel<<<std::min<unsigned>(grid_for(h->n, 256), 1024), 256, 0, h->stream>>>(
            h->n, h->x[c], h->y[c], h->th[c], h->dp.mark, h->dp.carry, d->tk[i] + 3 * kTicketWords,
            h->flags, d->scr[i], d->peers[i], step_io(h));
    }
    SLAM_HIP_TRY(hipGetLastError());
    int rc;
    for (int i = 0; i < m; ++i)                           // predict + likelihood
        if ((rc = launch_fused(d->sh[i], d->sh[i]->cfg.motion, false))) return rc;
    auto reduce = [&](int i, auto kern) {
        slam_pf* h = d->sh[i];
        const int c = h->cur;
        kern<<<1, kFinThreads, 0, h->stream>>>(
            h->n, h->dp, h->w_un, h->tail_leaves, h->tail_ops, h->n_tail_leaves, h->n_tail_ops,
            h->x[c], h->y[c], h->th[c], h->s_cur, h->refp, h->flags, h->cfg.ess_threshold,
            step_io(h), h->pc.np_recip, h->boff, d->scr[i], d->peers[i]);
    };
    if (m == 1) {                                         // record + push, wait, global finalize
        reduce(0, dist_reduce_kernel<true, true>);
    } else {                                              // one stream: every record first
        for (int i = 0; i < m; ++i) reduce(i, dist_reduce_kernel<true, false>);
        for (int i = 0; i < m; ++i) reduce(i, dist_reduce_kernel<false, true>);
    }
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

// ---- collective mode
hipStream_t dist_stream(slam_dist* d) { return d->local ? d->stream : d->sh[0]->stream; }

// rank r's slot [off + r bytes, + bytes) of every region into every region
int coll_all_gather(slam_dist* d, int64_t off, int64_t bytes) {
    hipStream_t s = dist_stream(d);
    if (d->comm) {
        char* reg = d->xbuf[0] + off;
        return comm_all_gather(d->comm->c, reg + (int64_t)d->rank0 * bytes, reg, (size_t)bytes, s);
    }
    for (int i = 0; i < d->nloc; ++i)
        for (int j = 0; j < d->nloc; ++j) {
            if (i == j) continue;
            const int64_t o = off + (int64_t)(d->rank0 + i) * bytes;
            SLAM_HIP_TRY(hipMemcpyAsync(d->xbuf[j] + o, d->xbuf[i] + o, (size_t)bytes,
                                        hipMemcpyDeviceToDevice, s));
        }
    return SLAM_OK;
}

// point-to-point: for every ordered pair (r -> q), q != r, bytes(r, q) from
// src(r, q) (in r's memory) to dst(q, r) (in q's memory)
template <typename Src, typename Dst, typename Bytes>
int coll_exchange(slam_dist* d, Src src, Dst dst, Bytes bytes) {
    hipStream_t s = dist_stream(d);
    if (d->comm) {
        const int r = d->rank0, w = d->world;
        std::vector<const void*> sp(w, nullptr);
        std::vector<void*> rp(w, nullptr);
        std::vector<size_t> sb(w, 0), rb(w, 0);
        for (int q = 0; q < w; ++q) {
            if (q == r) continue;
            sp[q] = src(0, q);
            sb[q] = (size_t)bytes(r, q);
            rp[q] = dst(0, q);
            rb[q] = (size_t)bytes(q, r);
        }
        return comm_exchange(d->comm->c, sp, sb, rp, rb, s);
    }
    for (int i = 0; i < d->nloc; ++i)
        for (int j = 0; j < d->nloc; ++j) {
            const int ri = d->rank0 + i, rj = d->rank0 + j;
            if (i == j || bytes(ri, rj) == 0) continue;
            SLAM_HIP_TRY(hipMemcpyAsync(dst(j, ri), src(i, rj), (size_t)bytes(ri, rj),
                                        hipMemcpyDeviceToDevice, s));
        }
    return SLAM_OK;
}

void coll_publish(slam_dist* d, int kind) {
    for (int i = 0; i < d->nloc; ++i) {
        slam_pf* h = d->sh[i];
        dist_publish_kernel<<<1, 64, 0, h->stream>>>(d->peers[i], kind, step_io(h));
    }
}

// One step with the exchanges as collectives between the launches (the
// kernels are the device-resident step's; their pushes stay in the own region
// or send area, and a publish launch stands for the peers' signals).  The
// host decides the resample branch from its mirror of the device flag and
// reads the specials' and items' counts it must move (two synchronisations
// on a resample step).
int dist_coll_step(slam_dist* d) {
    const int m = d->nloc, w = d->world;
    hipStream_t s = dist_stream(d);
    const DistLayout& L = d->L;
    const int64_t sz_spec = (int64_t)sizeof(SpecialIn), sz_item = (int64_t)sizeof(DistItem);
    int rc;
    if (d->sh[0]->resample_next) {
        for (int i = 0; i < m; ++i) {                     // exact cumsum: classify, emit (own slot)
            slam_pf* h = d->sh[i];
            const double delta = 4.0 * (double)h->n_global * 0x1p-53 + 0x1p-45;
            scan_classify_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
                h->w_un, h->n, h->boff, &d->scr[i]->base_off, h->c, h->kincl, h->fexcl, h->bk, h->bf,
                h->boffk, h->bofff, h->ktot, h->nspec, delta, h->gbase, h->tk + 2 * kTicketWords,
                h->flags, 0, h->s_cur, h->pc.np_recip, kPartPer);
        }
        for (int i = 0; i < m; ++i) {
            slam_pf* h = d->sh[i];
            dist_emit_push_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
                h->w_un, h->s_cur, h->pc.np_recip, h->n, h->c, h->kincl, h->fexcl, h->boffk, h->bofff,
                h->spec_in, h->gbase, h->nspec, h->ktot, d->tk[i], h->flags, d->peers[i], step_io(h));
        }
        // the specials: every rank's (count, increment total), then the lists
        if ((rc = coll_all_gather(d, L.spec_hdr, 16))) return rc;
        SLAM_HIP_TRY(hipMemcpyAsync(d->hst, d->xbuf[0] + L.spec_hdr, 16 * (size_t)w,
                                    hipMemcpyDeviceToHost, s));
        SLAM_HIP_TRY(hipStreamSynchronize(s));
        std::vector<int64_t> ns(w);
        for (int q = 0; q < w; ++q) ns[q] = std::min<int64_t>(std::max<int64_t>(d->hst[2 * q], 0), L.cap_spec);
        auto spec_slot = [&](int i, int q) { return d->xbuf[i] + L.spec + (int64_t)q * L.cap_spec * sz_spec; };
        if ((rc = coll_exchange(
                 d, [&](int i, int) { return (const void*)spec_slot(i, d->rank0 + i); },
                 [&](int j, int from) { return (void*)spec_slot(j, from); },
                 [&](int from, int) { return ns[from] * sz_spec; })))
            return rc;
        coll_publish(d, kXSpec);
        for (int i = 0; i < m; ++i) {                     // fold, expand + hi + counts, pack
            slam_pf* h = d->sh[i];
            dist_fold_kernel<<<1, 256, 0, h->stream>>>(d->spec_g[i], d->spec_go[i], h->n_global,
                                                       h->flags, d->scr[i], d->peers[i], step_io(h),
                                                       h->pc.rstep, h->pc.np_recip, h->cfg.seed);
        }
        for (int i = 0; i < m; ++i) {
            slam_pf* h = d->sh[i];
            dist_expand_hi_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
                h->n, h->kincl, h->fexcl, h->boffk, h->bofff, d->spec_go[i], h->c, d->hi[i], d->bsel[i],
                d->bsel_off[i], d->tk[i] + kTicketWords, h->flags, d->scr[i], d->peers[i], step_io(h),
                h->n_global, h->pc.rstep, h->pc.np_recip, h->cfg.seed);
        }
        for (int i = 0; i < m; ++i) {
            slam_pf* h = d->sh[i];
            const int c = h->cur;
            SLAM_HIP_TRY(hipMemsetAsync(d->peers[i].cnt_out, 0, 8 * (size_t)w, h->stream));
            dist_pack_push_kernel<<<h->nb_scan, kScanThreads, 0, h->stream>>>(
                h->n, h->x[c], h->y[c], h->th[c], d->hi[i], d->bsel_off[i], d->tk[i] + 2 * kTicketWords,
                h->flags, d->scr[i], d->peers[i], step_io(h));
        }
        // the items: every rank's counts per destination, then the items
        if (d->comm) {
            if ((rc = comm_all_gather(d->comm->c, d->peers[0].cnt_out, d->cnt_mat, 8 * (size_t)w, s)))
                return rc;
        } else {
            for (int i = 0; i < m; ++i)
                SLAM_HIP_TRY(hipMemcpyAsync(d->cnt_mat + (int64_t)(d->rank0 + i) * w, d->peers[i].cnt_out,
                                            8 * (size_t)w, hipMemcpyDeviceToDevice, s));
        }
        SLAM_HIP_TRY(hipMemcpyAsync(d->hst, d->cnt_mat, 8 * (size_t)w * w, hipMemcpyDeviceToHost, s));
        SLAM_HIP_TRY(hipStreamSynchronize(s));
        auto cnt = [&](int from, int to) {
            return std::min<int64_t>(std::max<int64_t>(d->hst[(int64_t)from * w + to], 0), L.cap_item);
        };
        // item headers of every held region (count from each source), then the items
        int64_t* hdr = d->hst + (int64_t)w * w;
        for (int i = 0; i < m; ++i) {
            int64_t* hi = hdr + 2 * (int64_t)w * i;
            for (int q = 0; q < w; ++q) {
                hi[2 * q] = cnt(q, d->rank0 + i);
                hi[2 * q + 1] = 0;
            }
            SLAM_HIP_TRY(hipMemcpyAsync(d->xbuf[i] + L.item_hdr, hi, 16 * (size_t)w, hipMemcpyHostToDevice,
                                        s));
        }
        if ((rc = coll_exchange(
                 d, [&](int i, int to) { return (const void*)(d->peers[i].item_out + (int64_t)to * L.cap_item); },
                 [&](int j, int from) {
                     return (void*)(d->xbuf[j] + L.item + (int64_t)from * L.cap_item * sz_item);
                 },
                 [&](int from, int to) { return cnt(from, to) * sz_item; })))
            return rc;
        coll_publish(d, kXItem);
        for (int i = 0; i < m; ++i) {
            slam_pf* h = d->sh[i];
            const int c = h->cur;
            dist_unpack_kernel<<<std::min<unsigned>(grid_for(h->n, 256), 1024), 256, 0, h->stream>>>(
                h->n, h->x[c], h->y[c], h->th[c], h->dp.mark, h->dp.carry, d->tk[i] + 3 * kTicketWords,
                h->flags, d->scr[i], d->peers[i], step_io(h));
        }
        SLAM_HIP_TRY(hipGetLastError());
    }
    for (int i = 0; i < m; ++i)                           // predict + likelihood
        if ((rc = launch_fused(d->sh[i], d->sh[i]->cfg.motion, false))) return rc;
    auto reduce = [&](int i, auto kern) {
        slam_pf* h = d->sh[i];
        const int c = h->cur;
        kern<<<1, kFinThreads, 0, h->stream>>>(
            h->n, h->dp, h->w_un, h->tail_leaves, h->tail_ops, h->n_tail_leaves, h->n_tail_ops,
            h->x[c], h->y[c], h->th[c], h->s_cur, h->refp, h->flags, h->cfg.ess_threshold,
            step_io(h), h->pc.np_recip, h->boff, d->scr[i], d->peers[i]);
    };
    for (int i = 0; i < m; ++i) reduce(i, dist_reduce_kernel<true, false>);      // records (own slot)
    const int par = (int)((d->sh[0]->stepno + 1) & 1);                         // dist_epoch parity
    if ((rc = coll_all_gather(d, L.g1 + (int64_t)par * w * L.rec_stride, L.rec_stride))) return rc;
    coll_publish(d, kXG1);
    for (int i = 0; i < m; ++i) reduce(i, dist_reduce_kernel<false, true>);      // global finalize
    SLAM_HIP_TRY(hipGetLastError());
    return SLAM_OK;
}

int dist_sync_results(slam_dist* d, int32_t first, int32_t count, slam_pf_result* out) {
    for (int i = 0; i < d->nloc; ++i) SLAM_HIP_TRY(hipStreamSynchronize(d->sh[i]->stream));
    int rc = sync_results(d->sh[0], first, count, out);
    for (int i = 0; i < count; ++i) {
        const int32_t st = d->sh[0]->res_host[first + i].status;
        if (st & kDistStWait) rc = fail(SLAM_ERR_COMM, "sharded step: a peer did not publish in time");
        if (st & kDistStItems) rc = fail(SLAM_ERR_COMM, "sharded resample: exchange inconsistent");
    }
    for (int i = 1; i < d->nloc; ++i) d->sh[i]->resample_next = d->sh[0]->resample_next;
    return rc;
}

// One captured hipGraph of `steps` sharded steps for the shards' current
// parity (slam_dist_run, slam_dist_prepare_graphs).
int dist_capture(slam_dist* d, hipGraphExec_t& ge, int steps) {
    hipStream_t s = d->sh[0]->stream;
    std::vector<int> cur0;
    for (auto* h : d->sh) cur0.push_back(h->cur);
    std::vector<char> timing0;                        // no timing events inside a graph
    for (auto* h : d->sh) {
        timing0.push_back(h->timing ? 1 : 0);
        h->timing = false;
    }
    hipGraph_t g;
    SLAM_HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = SLAM_OK;
    for (int k = 0; k < steps && rc == SLAM_OK; ++k) rc = dist_enqueue_step(d);
    const hipError_t e = hipStreamEndCapture(s, &g);
    for (int i = 0; i < d->nloc; ++i) {
        d->sh[i]->cur = cur0[i];
        d->sh[i]->timing = timing0[i] != 0;
    }
    if (rc) return rc;
    if (e != hipSuccess) return fail(SLAM_ERR_HIP, "slam_dist_run: hipStreamEndCapture failed");
    SLAM_HIP_TRY(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    SLAM_HIP_TRY(hipGraphUpload(ge, s));             // the first replay pays no upload
    return SLAM_OK;
}
}  // namespace

extern "C" {

int slam_pf_create_dist_shard(const slam_pf_config* cfg, int64_t n_local, int64_t n_global,
                              int64_t gbase, int32_t n_landmarks, const double* landmarks, int device,
                              slam_pf** out) {
    SLAM_ARG_CHECK(n_local % kSumChunk == 0 || gbase + n_local == n_global,
                   "slam_pf_create_dist_shard: every shard but the last must hold a multiple of "
                   "8192 particles (np.sum buffer alignment)");
    SLAM_ARG_CHECK(n_local <= (int64_t)2048 * kSumChunk, "slam_pf_create_dist_shard: n_local > 2^24");
    return create_impl(cfg, n_local, n_global, gbase, n_landmarks, landmarks, device, out, true, true);
}

// the standard split of N particles over `world` ranks: rank r holds
// [gbase, gbase + n_local); every shard but the last is a whole number of
// 8192-element np.sum buffers
int slam_dist_shard_range(int64_t n_global, int32_t world, int32_t rank, int64_t* gbase,
                          int64_t* n_local) {
    SLAM_ARG_CHECK(gbase && n_local && world >= 1 && rank >= 0 && rank < world && n_global >= world,
                   "slam_dist_shard_range: bad arguments");
    int64_t nf = (n_global + world - 1) / world;
    nf = (nf + kSumChunk - 1) / kSumChunk * kSumChunk;
    const int64_t g = std::min<int64_t>((int64_t)rank * nf, n_global);
    *gbase = g;
    *n_local = std::min<int64_t>(nf, n_global - g);
    return SLAM_OK;
}

int slam_dist_create(slam_pf** shards, int32_t n_held, int32_t world, int32_t rank0, slam_dist** out) {
    SLAM_ARG_CHECK(shards && out && n_held >= 1 && world >= 1 && world <= kDistMaxWorld &&
                       rank0 >= 0 && rank0 + n_held <= world,
                   "slam_dist_create: bad arguments");
    SLAM_ARG_CHECK(n_held == 1 || n_held == world,
                   "slam_dist_create: hold one shard (one process per GPU) or all of them (LOCAL)");
    *out = nullptr;
    const int64_t N = shards[0]->n_global;
    for (int i = 0; i < n_held; ++i) {
        SLAM_ARG_CHECK(shards[i] && shards[i]->deferred && shards[i]->n_global == N,
                       "slam_dist_create: shards must come from slam_pf_create_dist_shard, same filter");
        // the resample gathers address the staging slots either side of the
        // particle arrays (goff = npad), which only a dist shard has
        SLAM_ARG_CHECK(shards[i]->dp.goff > 0 &&
                           shards[i]->dp.goff == (int64_t)shards[i]->nb_part * kPartPer,
                       "slam_dist_create: handle is not a dist shard (slam_pf_create_dist_shard)");
        if (n_held > 1)
            SLAM_ARG_CHECK(shards[i]->device == shards[0]->device &&
                               (i == 0 ? shards[i]->gbase == 0
                                       : shards[i]->gbase == shards[i - 1]->gbase + shards[i - 1]->n),
                           "slam_dist_create: LOCAL shards must share one device and be contiguous");
    }
    if (n_held == world)
        SLAM_ARG_CHECK(shards[n_held - 1]->gbase + shards[n_held - 1]->n == N,
                       "slam_dist_create: the shards do not cover the filter");
    slam_dist* d = new slam_dist();
    d->world = world;
    d->rank0 = rank0;
    d->nloc = n_held;
    d->local = (n_held == world);
    d->device = shards[0]->device;
    d->sh.assign(shards, shards + n_held);
    // every failure from here on releases d and what it holds (slam_dist_destroy)
    auto bail = [&](int rc) {
        slam_dist_destroy(d);
        return rc;
    };
#define DIST_TRY(expr)                                                                    \
    do {                                                                                  \
        const hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess)                                                             \
            return bail(fail(SLAM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_))); \
    } while (0)
    DIST_TRY(hipSetDevice(d->device));
    // the largest shard sets the slot sizes (shards are equal but the last);
    // every rank must lay its region out the same way, so one shard per
    // process takes the standard split's full shard (rank 0's: ceil(N / world)
    // rounded up to whole np.sum buffers), not ceil(N / world) itself
    int64_t nmax = 0;
    for (auto* h : d->sh) nmax = std::max(nmax, h->n);
    if (!d->local) {
        int64_t g0 = 0, nfull = 0;
        slam_dist_shard_range(N, world, 0, &g0, &nfull);
        nmax = std::max<int64_t>(nmax, nfull);
    }
    const int64_t nch = (nmax + kSumChunk - 1) / kSumChunk;
    DistLayout& L = d->L;
    L.rec_stride = ((int64_t)sizeof(DistRec) + 8 * nch + 255) / 256 * 256;
    L.cap_spec = nmax;
    L.cap_item = nmax;
    int64_t off = 0;
    auto take = [&](int64_t bytes) {
        const int64_t o = off;
        off += (bytes + 4095) / 4096 * 4096;
        return o;
    };
    L.flags = take(3 * kDistMaxWorld * 8);
    L.g1 = take(2 * world * L.rec_stride);
    L.spec_hdr = take(16 * world);
    L.spec = take((int64_t)sizeof(SpecialIn) * L.cap_spec * world);
    L.item_hdr = take(16 * world);
    L.item = take((int64_t)sizeof(DistItem) * L.cap_item * world);
    L.pitem = take((int64_t)sizeof(DistRun) * L.cap_item);
    L.pcarry = take(8 * (L.cap_item / kPartPer + 2));
    L.total = off;
    int rc;
    if (d->local) {
        hipError_t e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
        if (e != hipSuccess) return bail(fail(SLAM_ERR_HIP, "slam_dist_create: stream creation failed"));
    }
    for (int i = 0; i < n_held; ++i) {
        slam_pf* h = d->sh[i];
        if (d->local && (rc = slam_pf_set_stream(h, d->stream, 1))) return bail(rc);
        void* xb = nullptr;
        if (hipExtMallocWithFlags(&xb, (size_t)L.total, hipDeviceMallocFinegrained) != hipSuccess)
            return bail(fail(SLAM_ERR_HIP, "slam_dist_create: fine-grained exchange region allocation failed"));
        d->xbuf.push_back((char*)xb);
        DIST_TRY(hipMemset(xb, 0, (size_t)L.flags + 3 * kDistMaxWorld * 8));
        // run tags (epoch >= 1) of the merged exchange start unmatched
        DIST_TRY(hipMemset((char*)xb + L.pitem, 0, (size_t)(L.total - L.pitem)));
        void *p1, *p2, *p3, *p4, *p5, *p6, *p7, *p8;
        const int32_t nbs = h->nb_scan;
        if ((rc = dist_alloc(d, &p1, sizeof(DistScratch))) ||
            (rc = dist_alloc(d, &p2, sizeof(SpecialIn) * (size_t)std::max<int64_t>(N, 1))) ||
            (rc = dist_alloc(d, &p3, sizeof(SpecialOut) * (size_t)std::max<int64_t>(N, 1))) ||
            (rc = dist_alloc(d, &p4, sizeof(int64_t) * (size_t)h->n)) ||
            (rc = dist_alloc(d, &p5, sizeof(int32_t) * (size_t)nbs)) ||
            (rc = dist_alloc(d, &p6, sizeof(int32_t) * (size_t)nbs)) ||
            (rc = dist_alloc(d, &p7, sizeof(unsigned) * 4 * kTicketWords)) ||
            (rc = dist_alloc(d, &p8, sizeof(DistItem) * (size_t)L.cap_item)))
            return bail(rc);
        DIST_TRY(hipMemset(p1, 0, sizeof(DistScratch)));
        DIST_TRY(hipMemset(p7, 0, sizeof(unsigned) * 4 * kTicketWords));
        d->scr.push_back((DistScratch*)p1);
        d->spec_g.push_back((SpecialIn*)p2);
        d->spec_go.push_back((SpecialOut*)p3);
        d->hi.push_back((int64_t*)p4);
        d->bsel.push_back((int32_t*)p5);
        d->bsel_off.push_back((int32_t*)p6);
        d->tk.push_back((unsigned*)p7);
        DistPeers P{};
        P.world = world;
        P.rank = rank0 + i;
        P.L = L;
        P.self_items = (DistItem*)p8;
        d->peers.push_back(P);
    }
    // shard bases.  LOCAL: the handles'.  One shard per process: the standard
    // split, n_full = ceil(N / world) rounded up to whole np.sum buffers, the
    // last rank taking the rest (slam_dist_shard_range)
    int64_t gb[kDistMaxWorld + 1];
    if (d->local) {
        for (int q = 0; q < world; ++q) gb[q] = d->sh[q]->gbase;
    } else {
        int64_t nf = 0;
        slam_dist_shard_range(N, world, 0, &gb[0], &nf);
        for (int q = 0; q < world; ++q) slam_dist_shard_range(N, world, q, &gb[q], &nf);
        int64_t g0 = 0, nl = 0;
        slam_dist_shard_range(N, world, rank0, &g0, &nl);
        if (d->sh[0]->gbase != g0 || d->sh[0]->n != nl)
            return bail(fail(SLAM_ERR_ARG, "slam_dist_create: shard is not slam_dist_shard_range's for its rank"));
    }
    gb[world] = N;
    {
        // one held shard: the resample exchange in one launch when its grid is
        // co-resident (its blocks wait for the last one twice); SLAM_DIST_MERGED=0
        // keeps the five-launch form
        int per_cu = 0, cus = 0;
        const char* ev = std::getenv("SLAM_DIST_MERGED");
        if (n_held == 1 && !(ev && ev[0] == '0') &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dist_resample_merged_kernel,
                                                         kScanThreads, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d->device) == hipSuccess)
            d->merged_ok = (int64_t)d->sh[0]->nb_scan <= (int64_t)per_cu * cus / 2;
        d->merged = d->merged_ok;
    }
    for (auto& P : d->peers)
        for (int q = 0; q <= world; ++q) P.gb[q] = gb[q];
    DIST_TRY(hipDeviceSynchronize());
#undef DIST_TRY
    if (d->local) {
        for (auto& P : d->peers)
            for (int q = 0; q < world; ++q) P.base[q] = d->xbuf[q];
        d->connected = true;
    }
    *out = d;
    return SLAM_OK;
}

// A rank's bootstrap blob: the IPC handle of its exchange region and the PCI
// bus id of its GPU (the peer-access preflight of slam_dist_connect).
constexpr int kDistBusId = 32;
constexpr size_t kDistBlob = sizeof(hipIpcMemHandle_t) + kDistBusId;

int slam_dist_handle_size(int64_t* bytes) {
    SLAM_ARG_CHECK(bytes, "slam_dist_handle_size: NULL argument");
    *bytes = (int64_t)kDistBlob;
    return SLAM_OK;
}

// bootstrap blobs of the held shards (n_held x slam_dist_handle_size bytes)
int slam_dist_export(slam_dist* d, void* blob) {
    SLAM_ARG_CHECK(d && blob, "slam_dist_export: NULL argument");
    SLAM_HIP_TRY(hipSetDevice(d->device));
    char bus[kDistBusId];
    std::memset(bus, 0, sizeof(bus));
    SLAM_HIP_TRY(hipDeviceGetPCIBusId(bus, kDistBusId - 1, d->device));
    for (int i = 0; i < d->nloc; ++i) {
        hipIpcMemHandle_t hd;
        SLAM_HIP_TRY(hipIpcGetMemHandle(&hd, d->xbuf[i]));
        char* b = (char*)blob + i * kDistBlob;
        std::memcpy(b, &hd, sizeof(hd));
        std::memcpy(b + sizeof(hd), bus, kDistBusId);
    }
    return SLAM_OK;
}

// every rank's handle (world x handle size, rank order): open the peers'
int slam_dist_connect(slam_dist* d, const void* all_blobs) {
    SLAM_ARG_CHECK(d && all_blobs, "slam_dist_connect: NULL argument");
    if (d->connected) return SLAM_OK;
    SLAM_HIP_TRY(hipSetDevice(d->device));
    // preflight: every peer's GPU reachable from this one (the exchange stores
    // into peer memory over xGMI); fail loudly instead of in the first wait
    for (int q = 0; q < d->world; ++q) {
        if (q >= d->rank0 && q < d->rank0 + d->nloc) continue;
        char bus[kDistBusId];
        std::memcpy(bus, (const char*)all_blobs + q * kDistBlob + sizeof(hipIpcMemHandle_t), kDistBusId);
        bus[kDistBusId - 1] = 0;
        int dev = -1;
        if (hipDeviceGetByPCIBusId(&dev, bus) != hipSuccess || dev < 0)
            return fail(SLAM_ERR_COMM, std::string("slam_dist_connect: rank ") + std::to_string(q) +
                                           "'s GPU (PCI " + bus + ") is not visible to this process");
        if (dev == d->device) continue;                  // ranks sharing one GPU
        int can = 0;
        SLAM_HIP_TRY(hipDeviceCanAccessPeer(&can, d->device, dev));
        if (!can)
            return fail(SLAM_ERR_COMM, std::string("slam_dist_connect: no peer access from device ") +
                                           std::to_string(d->device) + " to rank " + std::to_string(q) +
                                           "'s device " + std::to_string(dev) + " (PCI " + bus + ")");
    }
    std::vector<char*> base(d->world, nullptr);
    for (int q = 0; q < d->world; ++q) {
        if (q >= d->rank0 && q < d->rank0 + d->nloc) {
            base[q] = d->xbuf[q - d->rank0];
            continue;
        }
        hipIpcMemHandle_t hd;
        std::memcpy(&hd, (const char*)all_blobs + q * kDistBlob, sizeof(hd));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, hd, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess)
            return fail(SLAM_ERR_COMM, std::string("hipIpcOpenMemHandle (peer exchange region): ") +
                                           hipGetErrorString(e));
        d->opened.push_back(p);
        base[q] = (char*)p;
    }
    for (auto& P : d->peers)
        for (int q = 0; q < d->world; ++q) P.base[q] = base[q];
    d->connected = true;
    return SLAM_OK;
}

// one-call bootstrap over an RCCL communicator (rank = comm rank)
int slam_dist_connect_comm(slam_dist* d, slam_comm* comm) {
    SLAM_ARG_CHECK(d && comm && d->nloc == 1, "slam_dist_connect_comm: one held shard per process");
    int32_t w = 0, r = 0;
    int rc = slam_comm_info(comm, &w, &r);
    if (rc) return rc;
    SLAM_ARG_CHECK(w == d->world && r == d->rank0, "slam_dist_connect_comm: communicator rank mismatch");
    const size_t hs = kDistBlob;
    std::vector<char> mine(hs), all(hs * w);
    if ((rc = slam_dist_export(d, mine.data()))) return rc;
    if ((rc = slam_comm_all_gather_host(comm, mine.data(), all.data(), (int64_t)hs))) return rc;
    return slam_dist_connect(d, all.data());
}

// Exchange by collectives instead of peer-memory stores (the fallback when a
// peer's exchange region cannot be mapped): one held shard with an RCCL
// communicator of the filter's world (rank = comm rank), or every shard held
// (LOCAL) with comm = NULL -- the collectives are then device copies between
// the held regions.  The steps become host-orchestrated (no hipGraphs).
int slam_dist_set_collective(slam_dist* d, slam_comm* comm) {
    SLAM_ARG_CHECK(d, "slam_dist_set_collective: NULL handle");
    if (comm) {
        int32_t w = 0, r = 0;
        int rc = slam_comm_info(comm, &w, &r);
        if (rc) return rc;
        SLAM_ARG_CHECK(d->nloc == 1 && w == d->world && r == d->rank0,
                       "slam_dist_set_collective: one held shard, communicator of the filter's world and rank");
    } else {
        SLAM_ARG_CHECK(d->local, "slam_dist_set_collective: without a communicator every shard must be held");
    }
    SLAM_HIP_TRY(hipSetDevice(d->device));
    dist_drop_graphs(d);
    const int w = d->world;
    if (!d->cnt_mat) {
        void* p = nullptr;
        int rc = dist_alloc(d, &p, 8 * (size_t)w * w);
        if (rc) return rc;
        d->cnt_mat = (int64_t*)p;
        SLAM_HIP_TRY(hipHostMalloc((void**)&d->hst, 8 * (size_t)(3 * w * w + 16)));
        for (int i = 0; i < d->nloc; ++i) {
            void *io = nullptr, *co = nullptr;
            if ((rc = dist_alloc(d, &io, sizeof(DistItem) * (size_t)w * (size_t)d->L.cap_item)) ||
                (rc = dist_alloc(d, &co, 8 * (size_t)w)))
                return rc;
            d->peers[i].item_out = (DistItem*)io;
            d->peers[i].cnt_out = (int64_t*)co;
        }
    }
    for (int i = 0; i < d->nloc; ++i) {
        DistPeers& P = d->peers[i];
        P.coll = 1;
        for (int q = 0; q < w; ++q) P.base[q] = (q == d->rank0 + i) ? d->xbuf[i] : nullptr;
    }
    // the shards' flag words start over (the epochs published by publish launches)
    for (int i = 0; i < d->nloc; ++i)
        SLAM_HIP_TRY(hipMemset(d->xbuf[i] + d->L.flags, 0, 3 * kDistMaxWorld * 8));
    d->comm = comm;
    d->coll = true;
    d->merged = false;
    d->connected = true;
    return SLAM_OK;
}

int slam_dist_destroy(slam_dist* d) {
    if (!d) return SLAM_OK;
    (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    for (auto* h : d->sh)
        if (h && h->stream) (void)hipStreamSynchronize(h->stream);
    dist_drop_graphs(d);
    for (void* p : d->opened) (void)hipIpcCloseMemHandle(p);
    if (d->hst) (void)hipHostFree(d->hst);
    for (char* p : d->xbuf) (void)hipFree(p);
    for (void* p : d->dallocs) (void)hipFree(p);
    // LOCAL: the shards keep running on private streams again
    if (d->local)
        for (auto* h : d->sh)
            if (h) (void)slam_pf_set_stream(h, nullptr, 0);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
    return SLAM_OK;
}

// One step of every held shard (device RNG noise and resample offset; the
// observations of this step staged in slot 0).  res: the global result
// (identical on every rank).
// one-launch (1) or five-launch (0) resample exchange; reports the form in use
int slam_dist_set_merged(slam_dist* d, int32_t on, int32_t* active) {
    SLAM_ARG_CHECK(d, "slam_dist_set_merged: NULL handle");
    if (on >= 0) {
        SLAM_ARG_CHECK(!on || (d->merged_ok && !d->coll),
                       "slam_dist_set_merged: needs one held shard with a co-resident scan grid "
                       "(and the peer-memory exchange)");
        if (d->merged != (on != 0)) dist_drop_graphs(d);
        d->merged = on != 0;
    }
    if (active) *active = d->merged ? 1 : 0;
    return SLAM_OK;
}

int slam_dist_step(slam_dist* d, const double* control, const double* z, slam_pf_result* res) {
    SLAM_ARG_CHECK(d && control && d->connected, "slam_dist_step: bad argument or not connected");
    SLAM_HIP_TRY(hipSetDevice(d->device));
    int rc;
    for (auto* h : d->sh)
        if ((rc = stage_inputs(h, control, z, nullptr, std::nan("")))) return rc;
    if ((rc = d->coll ? dist_coll_step(d) : dist_enqueue_step(d))) return rc;
    for (auto* h : d->sh) h->stepno++;
    return dist_sync_results(d, 0, 1, res);
}

int slam_dist_load_observations(slam_dist* d, int32_t n_steps, const double* z_all) {
    SLAM_ARG_CHECK(d, "slam_dist_load_observations: NULL handle");
    dist_drop_graphs(d);
    for (auto* h : d->sh) {
        const int rc = slam_pf_load_observations(h, n_steps, z_all);
        if (rc) return rc;
    }
    return SLAM_OK;
}

// n_steps device-resident steps from loaded observations, replayed as
// captured hipGraphs (kGraphSteps per graph); results of the first held shard.
int slam_dist_run(slam_dist* d, int32_t first_step, int32_t n_steps, const double* controls,
                  slam_pf_result* results) {
    SLAM_ARG_CHECK(d && controls && n_steps > 0 && d->connected, "slam_dist_run: bad argument");
    SLAM_HIP_TRY(hipSetDevice(d->device));
    for (auto* h : d->sh) {
        SLAM_ARG_CHECK(first_step >= 0 && first_step + n_steps <= h->z_steps,
                       "slam_dist_run: steps outside the loaded observations");
        // controls, counters and the first step's closed-form words (the
        // exchange owns the resample flag)
        const int rc = launch_run_setup(h, first_step, n_steps, controls, -1);
        if (rc) return rc;
    }
    int rc;
    if (d->coll) {                             // host-orchestrated steps, one result read each
        for (int32_t k = 0; k < n_steps; ++k) {
            if ((rc = dist_coll_step(d))) return rc;
            for (auto* h : d->sh) h->stepno++;
            if ((rc = dist_sync_results(d, first_step + k, 1, nullptr))) return rc;
        }
        return dist_sync_results(d, first_step, n_steps, results);
    }
    const bool graphs = d->sh[0]->use_graph && !d->sh[0]->timing;
    hipStream_t s = d->sh[0]->stream;          // LOCAL: the shared stream; else the shard's
    int32_t k = 0;
    while (k < n_steps) {
        const int par = d->sh[0]->cur;
        if (graphs) {
            const bool multi = n_steps - k >= kGraphSteps;
            hipGraphExec_t& ge = multi ? d->graph[par] : d->graph1[par];
            if (!ge && (rc = dist_capture(d, ge, multi ? kGraphSteps : 1))) return rc;
            SLAM_HIP_TRY(hipGraphLaunch(ge, s));
            const int done = multi ? kGraphSteps : 1;
            if (done & 1)
                for (auto* h : d->sh) h->cur = 1 - h->cur;
            k += done;
            for (auto* h : d->sh) h->stepno += done;
        } else {
            if ((rc = dist_enqueue_step(d))) return rc;
            ++k;
            for (auto* h : d->sh) h->stepno++;
        }
    }
    return dist_sync_results(d, first_step, n_steps, results);
}

int slam_dist_prepare_graphs(slam_dist* d, double* capture_ms) {
    SLAM_ARG_CHECK(d && d->connected, "slam_dist_prepare_graphs: bad argument");
    SLAM_HIP_TRY(hipSetDevice(d->device));
    const auto t0 = std::chrono::steady_clock::now();
    int rc = SLAM_OK;
    if (d->sh[0]->use_graph && !d->coll) {
        std::vector<int> cur0;
        for (auto* h : d->sh) cur0.push_back(h->cur);
        for (int par = 0; par < 2 && rc == SLAM_OK; ++par) {
            for (auto* h : d->sh) h->cur = par;
            if (!d->graph[par]) rc = dist_capture(d, d->graph[par], kGraphSteps);
            if (!rc && !d->graph1[par]) rc = dist_capture(d, d->graph1[par], 1);
        }
        for (int i = 0; i < d->nloc; ++i) d->sh[i]->cur = cur0[i];
    }
    if (capture_ms)
        *capture_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

}  // extern "C"

// --use-ars: exact association rules between frequent conditions (included by kernels.inl).
//
// FrequentConditionPlanner.findAssociationRules (ALG/plan/FrequentConditionPlanner.scala:130-194): a frequent binary
// condition (a=va, c=vc) whose triple count equals the count of its unary condition a=va yields the rule
// a=va -> c=vc (confidence 1, the only rules kept, :186-190).  Binary keys: bt 0 = (p, o), 1 = (s, o), 2 = (s, p),
// v1 the value at the lower position, so every key can give the rule lower -> upper and upper -> lower.
// Consumers: CreateJoinPartners drops the AR-implied binary captures (CreateJoinPartners.scala:99-141,
// isAssociationRuleImplied :161-171), and the 1/1 CIND A < B of every rule is never produced
// (CreateAllCindCandidates.scala:108-115; SmallToLargeTraversalStrategy.scala:80-85).

// condition positions (0 s, 1 p, 2 o) of binary key type bt
__host__ __device__ inline void bin_key_positions(int bt, int& pa, int& pb) {
    pa = bt == 0 ? 1 : 0;
    pb = bt == 2 ? 1 : 2;
}

// triple counts of the frequent unary conditions (by global rank) and of the frequent binary conditions (by index b);
// equal keys of a wave merge first (hot predicates), one atomic per distinct key per wave
__global__ __launch_bounds__(RDF_BLOCK) void k_ar_count(const u32* __restrict__ s, const u32* __restrict__ p,
                                                        const u32* __restrict__ o, u64 n, u32 V,
                                                        const u32* __restrict__ frank, const u64* __restrict__ lkeys,
                                                        const u32* __restrict__ lvals, u64 lmask, u32* ucnt, u32* bcnt) {
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    const u64 b = (u64)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (u64 i0 = b; i0 < e; i0 += RDF_BLOCK) {
        const u64 i = i0 + threadIdx.x;
        const bool act = i < e;
        const u32 ts = act ? s[i] : 0u, tp = act ? p[i] : 0u, to = act ? o[i] : 0u;
        const u32 r[3] = {act ? frank[ts] : NONE32, act ? frank[(u64)V + tp] : NONE32, act ? frank[2ull * V + to] : NONE32};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32 c = wave_merge_weighted<u32, 4>(r[k], r[k] != NONE32, 1u);
            if (c) atomicAdd(&ucnt[r[k]], c);
        }
        u32 bk[3];
        bk[0] = (r[1] != NONE32 && r[2] != NONE32) ? bin_lookup(lkeys, lvals, lmask, bin_key(0, tp, to)) : NONE32;
        bk[1] = (r[0] != NONE32 && r[2] != NONE32) ? bin_lookup(lkeys, lvals, lmask, bin_key(1, ts, to)) : NONE32;
        bk[2] = (r[0] != NONE32 && r[1] != NONE32) ? bin_lookup(lkeys, lvals, lmask, bin_key(2, ts, tp)) : NONE32;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32 c = wave_merge_weighted<u32, 4>(bk[k], bk[k] != NONE32, 1u);
            if (c) atomicAdd(&bcnt[bk[k]], c);
        }
    }
}

// rule bits of frequent binary key b (bit 0: lower -> upper, bit 1: upper -> lower), their popcount (rule slots)
// and the keep flag of the key (no rule: the binary capture stays)
__global__ __launch_bounds__(RDF_BLOCK) void k_ar_flags(const u64* __restrict__ bkeys, u64 B, u32 V,
                                                        const u32* __restrict__ frank, const u32* __restrict__ ucnt,
                                                        const u32* __restrict__ bcnt, u32* rbits, u32* nrule, u32* keep) {
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b < B; b += (u64)gridDim.x * RDF_BLOCK) {
        const u64 key = bkeys[b];
        int pa, pb;
        bin_key_positions(bin_key_type(key), pa, pb);
        const u32 cb = bcnt[b];
        const u32 ca = ucnt[frank[(u64)pa * V + bin_key_v1(key)]];
        const u32 cc = ucnt[frank[(u64)pb * V + bin_key_v2(key)]];
        const u32 r = (ca == cb ? 1u : 0u) | (cc == cb ? 2u : 0u);
        rbits[b] = r;
        nrule[b] = (u32)__popc(r);
        keep[b] = r ? 0u : 1u;
    }
}

// rules of key b at rpos[b]: (antecedent type, consequent type, antecedent, consequent, support) with condition
// codes s = 1, p = 2, o = 4 (ConditionCodes); the kept keys are compacted to kout at kpos[b]
__global__ __launch_bounds__(RDF_BLOCK) void k_ar_emit(const u64* __restrict__ bkeys, u64 B, const u32* __restrict__ rbits,
                                                       const u32* __restrict__ bcnt, const u32* __restrict__ rpos,
                                                       const u32* __restrict__ kpos, u32* rules, u64* kout) {
    for (u64 b = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; b < B; b += (u64)gridDim.x * RDF_BLOCK) {
        const u64 key = bkeys[b];
        const u32 r = rbits[b];
        if (!r) {
            kout[kpos[b]] = key;
            continue;
        }
        int pa, pb;
        bin_key_positions(bin_key_type(key), pa, pb);
        const u32 v1 = bin_key_v1(key), v2 = bin_key_v2(key), cb = bcnt[b];
        u32* w = rules + 5ull * rpos[b];
        if (r & 1u) {
            w[0] = 1u << pa; w[1] = 1u << pb; w[2] = v1; w[3] = v2; w[4] = cb;
            w += 5;
        }
        if (r & 2u) {
            w[0] = 1u << pb; w[1] = 1u << pa; w[2] = v2; w[3] = v1; w[4] = cb;
        }
    }
}

// AR-implied 1/1 CIND of each rule (FilterAssociationRuleImpliedCinds.AssocationRuleBroadcastInitializer,
// FilterAssociationRuleImpliedCinds.scala:44-58): rule a -> c at the third position pi gives pi[a] < pi[c].
// arref[compact id of pi[a]] = compact id of pi[c] when both captures are frequent (unique per dependent: the
// triples of a=va all carry the same consequent value).  Unary candidate id = 2 * rank + j, j = 1 when the
// projection is the higher of the two positions other than the condition's (ucap).
__global__ __launch_bounds__(RDF_BLOCK) void k_ar_refs(const u32* __restrict__ rules, u64 nr, u32 V,
                                                       const u32* __restrict__ frank, const u32* __restrict__ support,
                                                       const u32* __restrict__ fidx, u32 ms, u32* arref) {
    for (u64 i = (u64)blockIdx.x * RDF_BLOCK + threadIdx.x; i < nr; i += (u64)gridDim.x * RDF_BLOCK) {
        const u32* w = rules + 5 * i;
        const int pa = __ffs(w[0]) - 1, pc = __ffs(w[1]) - 1;
        const int pi = 3 - pa - pc;
        const u32 ja = pi > 3 - pa - pi ? 1u : 0u, jc = pi > 3 - pc - pi ? 1u : 0u;
        const u32 da = 2u * frank[(u64)pa * V + w[2]] + ja;
        const u32 dc = 2u * frank[(u64)pc * V + w[3]] + jc;
        if (support[da] >= ms && support[dc] >= ms) arref[fidx[da]] = fidx[dc];
    }
}

// --use-ars on the discovery side (DESIGN.md "Association rules"): CINDs the reference never produces.
//   both strategies: the 1/1 CIND A < arref[A] (CreateAllCindCandidates.scala:108-115 leaves the AR-implied ref
//   out of A's candidates; S2L filters its 1/1 CINDs, SmallToLargeTraversalStrategy.scala:80-85);
//   S2L only, whose larger candidates are built from the filtered 1/1 CINDs:
//     1/2 A < X when A implies a component of X (no 1/1 pair to generate X from,
//       GenerateUnaryBinaryCindCandidates, SmallToLargeTraversalStrategy.scala:368-376);
//     2/2 D < Y when a component of Y outside D is implied by a component of D (D < Yk is neither a proper-overlap
//       2/1 candidate nor inferred from a kept 1/1 CIND, InferDoubleSingleCinds, SmallToLargeTraversalStrategy.scala:497-562).
__device__ inline bool ar_drop(const CindView& v, u32 d, u32 r) {
    if (!v.ar) return false;
    if (d < v.Cu) {
        const u32 a = v.arref[d];
        if (a == NONE32) return false;
        if (r < v.Cu) return a == r;
        if (v.ar != AR_S2L) return false;
        const u32* rc = v.bcomp + 2ull * (r - v.Cu);
        return a == rc[0] || a == rc[1];
    }
    if (v.ar != AR_S2L || r < v.Cu) return false;
    const u32* dc = v.bcomp + 2ull * (d - v.Cu);
    const u32* rc = v.bcomp + 2ull * (r - v.Cu);
    const u32 a0 = v.arref[dc[0]], a1 = v.arref[dc[1]];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const u32 y = rc[k];
        if (y != dc[0] && y != dc[1] && (a0 == y || a1 == y)) return true;
    }
    return false;
}

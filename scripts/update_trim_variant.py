# Generates the trimmed k_update variants of profiles/r03_ab_update_waves.txt
# (python3 scripts/update_trim_variant.py TAG [smin] [lb4] -> fast-slam_amd/csrc/fuvTAG.hip;
# swap it in for fs2_update.hip to build an A/B library, then restore).
import sys
s=open('fast-slam_amd/csrc/fs2_update.hip').read()
def rep(old,new):
    global s
    assert old in s, old[:80]
    s=s.replace(old,new)
i=s.index('''    } else {
        // An overflowing list: the reference's loop''')
j=s.index('''    FS2_PHASE(2);''')
s=s[:i]+'''    }
'''+s[j:]
rep('''            s_lik[k][tid] = ekf_update(s, px, py, pyaw, mk, R, singular);
            const float4 mv = store_slot(map, pg, jh, s, r, jh);''','''            s_lik[k][tid] = 1.0;
            const float4 mv = store_slot(map, pg, jh, s, r, jh);''')
rep('''        uint64_t e0 = entry(0), e1 = entry(1);
        Slot s0 = load_rec(map.recs, rec_of(0, e0));
        for (int p = 0; p < nl && pend != 0u; ++p) {
            const uint64_t e2 = entry(p + 2);
            const Slot s1 = load_rec(map.recs, rec_of(p + 1, e1));
            visit(cand_slot(e0), cand_pos(e0), s0);
            e0 = e1;
            s0 = s1;
            e1 = e2;
        }''','''        for (int p = 0; p < nl && pend != 0u; ++p) {
            const uint64_t e0 = entry(p);
            visit(cand_slot(e0), cand_pos(e0), load_rec(map.recs, rec_of(p, e0)));
        }''')
rep('''    uint32_t frec[MAXM];
#pragma unroll
    for (int t = 0; t < MAXM; ++t) {
        frec[t] = (live && t < P.m) ? P.alloc.rfreel[P.alloc.rbase + (int64_t)t * n + i] : 0u;
    }''','''    auto frec_at = [&](int t) -> uint32_t { return P.alloc.rfreel[P.alloc.rbase + (int64_t)t * n + il]; };''')
s=s.replace('sel_u32(nmod, frec)','frec_at(nmod)').replace('sel_u32(nrec, frec)','frec_at(nrec)').replace('sel_u32(q, frec)','frec_at(q)').replace('sel_u32(t2, frec)','frec_at(t2)')
rep('''        w = P.w[i];
        c = P.cnt[i];''','''        c = P.cnt[i];''')
rep('''    unsigned hits = 0, refv = 0, napp = 0;''','''    unsigned hits = 0, refv = 0, napp = 0;
    if (live) w = P.w[i];''')
if 'smin' in sys.argv:
    rep('''            smin_w = fminf(smin_w, mirror_s(m) > 0.0f ? mirror_s(m) : INFINITY);
            s_mv[nmod][tid] = m;''','''            s_mv[nmod][tid] = m;''')
    rep('''                reinterpret_cast<float4 *>(page_ptr(map.pool, id))[j & (kPageSlots - 1)] = s_mv[t][tid];''','''                const float4 mvt = s_mv[t][tid];
                smin_w = fminf(smin_w, mirror_s(mvt) > 0.0f ? mirror_s(mvt) : INFINITY);
                reinterpret_cast<float4 *>(page_ptr(map.pool, id))[j & (kPageSlots - 1)] = mvt;''')
if 'lb4' in sys.argv:
    s=s.replace('__launch_bounds__(kBlock, FS2_UPDATE_WAVES) void k_update','__launch_bounds__(kBlock, 4) void k_update')
open('fast-slam_amd/csrc/fuv%s.hip'%sys.argv[1],'w').write(s)

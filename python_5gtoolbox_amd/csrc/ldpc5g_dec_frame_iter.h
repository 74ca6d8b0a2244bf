// ldpc5g_dec_frame_iter.h — the decode iterations of frame_body (ldpc5g_dec_frame.h), included
// inside it twice by a workgroup-uniform choice: with DEAD = true (the dead-extension-row
// shortcuts, for a codeblock with a dead row) and DEAD = false.  A textual include rather than a
// generic lambda: the lambda form spills VGPRs in the plain kernel (measured ~1 % slower).
// No include guard on purpose; not a standalone header.

    auto rdead = [&](int i) -> bool { return DEAD && i >= 4 && ((live_x >> (i - 4)) & 1u) == 0; };
    for (; it < L; ++it) {
        // opaque per iteration: otherwise LICM hoists hundreds of loop-invariant addresses
        uint32_t sb = sb0, sbw = sbw0, tz = tz0;
        int sv = s;
        asm volatile("" : "+v"(sb));
        asm volatile("" : "+v"(sbw));
        asm volatile("" : "+v"(tz));
        asm volatile("" : "+v"(sv));
        auto rot = [&](int c) -> uint32_t { return fr_rot(sb, sbw, c); };
        // check node of row i run by this thread: (s - off[i]) mod Zc
        auto xpos = [&](int i) -> int {
            const int c = (Z - kFrPlan<BG>.off[i]) % Z;
            if (c == 0) return sv;
            return (int)min((uint32_t)(sv + c), (uint32_t)(sv + c - Z));
        };
        auto llrx = [&](int i) -> T { return ldg(lrow_x, i * Z + xpos(i)); };
        bool fail = false;
        uint64_t hdx = 0;   // hard decisions of the owned extension columns (LQ_old)

        // ext LLR ring: slot p % XP holds the LLR of the half's ext row p, loaded XP rows ahead
        constexpr int XP = kXPre > 0 ? kXPre : 1;
        T xr[XP];
        auto xload = [&](auto hc, auto pc_) {
            constexpr int hh = decltype(hc)::value, p = decltype(pc_)::value;
            if constexpr (p < kFrPlan<BG>.nx[hh]) xr[p % XP] = llrx(kFrPlan<BG>.xlist[hh][p]);
        };
        // ---- phase A: new row state from LQ_old (:117-123, _min_sum_process :186-202).  The
        // half's core-edge stream (FrStream): entry p's wrap-table offset is read kFrDT positions
        // ahead and its LQ kFrDA ahead, across row boundaries (slots p % kFrDT, p % kFrDA)
        struct RowSt {
            T mA, mB, min1, min2;
            uint32_t u, idxo, idx, negs;
            bool par;
        };
        uint32_t tbs[kFrDT];
        T abq[kFrDA];
        auto sload_t = [&](auto hc, auto pc_) {
            constexpr int hh = decltype(hc)::value, p = decltype(pc_)::value;
            if constexpr (p < kFrStr<BG>.n[hh]) {
                constexpr int i = kFrStr<BG>.row[hh][p], k = kFrStr<BG>.k[hh][p];
                tbs[p % kFrDT] = *(lds_u32*)(uintptr_t)(tz + (uint32_t)fr_cof<BG>(i, k) * 4u);
            }
        };
        auto sload_a = [&](auto hc, auto pc_) {
            constexpr int hh = decltype(hc)::value, p = decltype(pc_)::value;
            if constexpr (p < kFrStr<BG>.n[hh]) {
                constexpr int i = kFrStr<BG>.row[hh][p], k = kFrStr<BG>.k[hh][p];
                abq[p % kFrDA] = at((uint32_t)(P::COL[P::RS[i] + k] * kFrColB) + tbs[p % kFrDT]);
            }
        };
        // core edge k of row i: its LQ entry, and the stream moved on by one
        auto snext = [&](auto ic, auto kc) -> T {
            constexpr int i = decltype(ic)::value, k = decltype(kc)::value;
            constexpr int hh = kFrPlan<BG>.owner[i], p = kFrStr<BG>.start[i] + k;
            const T a = abq[p % kFrDA];
            sload_a(std::integral_constant<int, hh>{}, std::integral_constant<int, p + kFrDA>{});
            sload_t(std::integral_constant<int, hh>{}, std::integral_constant<int, p + kFrDT>{});
            return a;
        };
        auto rowA = [&](auto ic) {
            constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = kFrPlan<BG>.deg(i);
            RowSt r;
            get_state(ic, r.mA, r.mB, r.u, r.idxo);
            r.min1 = FT<T>::inf(), r.min2 = FT<T>::inf();
            r.idx = 0, r.negs = 0, r.par = false;
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value, j = P::COL[e0 + k];
                const T rold = xsign_v(pick(r.idxo == (uint32_t)k, r.mB, r.mA), r.u, mv);
                asm("v_add_u32 %0, %1, %1" : "=v"(r.u) : "v"(r.u));   // u <<= 1, all-VGPR form
                T a;
                if constexpr (j < KC) {
                    a = snext(ic, kc);
                    __builtin_amdgcn_sched_barrier(0);
                    r.par ^= a < T(0);
                } else {
                    constexpr int hh = kFrPlan<BG>.owner[i], p = kFrPlan<BG>.xpos[i];
                    a = xr[p % XP] + rold;   // LQ of a degree-1 column = LLR + its only r
                    xload(std::integral_constant<int, hh>{}, std::integral_constant<int, p + XP>{});
                    hdx |= (uint64_t)(a < T(0)) << (i - 4);
                    r.par ^= a < T(0);
                }
                const T q = a - rold;
                const T aq = fabs(q);
                r.idx = aq < r.min1 ? (uint32_t)k : r.idx;
                asm volatile("" : "+v"(r.idx));
                r.negs = __builtin_amdgcn_alignbit(r.negs, FT<T>::sbits(q), 31);
                two_min(r.min1, r.min2, aq);
            });
            fail |= r.par;
            T x1 = r.min1, x2 = r.min2;
            if constexpr (OFS) {
                x1 = r.min1 - beta, x2 = r.min2 - beta;   // max(minv - beta, 0) (:201)
                x1 = x1 > T(0) ? x1 : T(0), x2 = x2 > T(0) ? x2 : T(0);
            }
            const uint32_t sgn = 0u - (__builtin_popcount(r.negs) & 1u);   // the row's sign product
            put_state(ic, alpha * x1, alpha * x2, r.negs ^ (sgn & ((1u << d) - 1u)), r.idx);
        };
        // a dead extension row: LQ_ext = 0 + r_old_ext (its syndrome bit), q_core = LQ - (+-0); the
        // new state as the full update leaves it up to zero signs (ldpc5g_dec_flood.h rowA_dead)
        auto rowA_dead = [&](auto ic) {
            constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = kFrPlan<BG>.deg(i);
            T mA, mB;
            uint32_t u, idxo;
            get_state(ic, mA, mB, u, idxo);
            const T rext = xsign_v(pick(idxo == (uint32_t)(d - 1), mB, mA), u << (d - 1), mv);
            constexpr int hh = kFrPlan<BG>.owner[i], p = kFrPlan<BG>.xpos[i];
            xload(std::integral_constant<int, hh>{}, std::integral_constant<int, p + XP>{});   // keep the ring moving
            const T ax = T(0) + rext;
            hdx |= (uint64_t)(ax < T(0)) << (i - 4);
            bool par = ax < T(0);
            T mn = FT<T>::inf();
            uint32_t sx = 0;
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value, j = P::COL[e0 + k];
                if constexpr (j < KC) {
                    const T a = snext(ic, kc);
                    par ^= a < T(0);
                    mn = fmin(mn, fabs(a));
                    sx ^= FT<T>::sbits(a);
                }
            });
            fail |= par;
            T x2 = mn;
            if constexpr (OFS) {
                x2 = mn - beta;
                x2 = x2 > T(0) ? x2 : T(0);
            }
            put_state(ic, T(0), alpha * x2, sx >> 31, (uint32_t)(d - 1));
        };
        if (active) {
            per_half([&](auto hc) {
                sfor<0, XP>([&](auto pc_) { xload(hc, pc_); });
                sfor<0, kFrDT>([&](auto pc_) { sload_t(hc, pc_); });
                sfor<0, kFrDA>([&](auto pc_) { sload_a(hc, pc_); });
            });
            sfor<0, MB>([&](auto ic) {   // one branch per row: bounded live ranges
                constexpr int i = decltype(ic)::value;
                if (h == kFrPlan<BG>.owner[i]) {
                    if constexpr (DEAD && i >= 4) {
                        if (rdead(i)) rowA_dead(ic);
                        else rowA(ic);
                    } else {
                        rowA(ic);
                    }
                }
            });
            if (fail) *flagA = 1;
        }
        lds_barrier();
        // ---- the syndrome of LQ_old decides (:107-114): output its hard decisions
        if (active && *flagA == 0) {
            hdx_keep = hdx;   // the LQ image stays frozen (no phase B) for the decisions
            if (t == 0) status[out] = 1, iters[out] = it;
            active = false;
        }

        // ---- phase B: Lr.sum(axis=0) in row order (:126).  Columns >= 2: ds_add into the LQ
        // image, one barrier per group; column h: this thread's register sum S.
        auto msg = [&](T a, T b, uint32_t u, uint32_t idx, auto kc) -> T {   // r of edge k
            constexpr int k = decltype(kc)::value;
            return xsign_v(pick(idx == (uint32_t)k, b, a), u << k, mv);
        };
        auto add_to = [&](auto ic, auto kc, T r, uint32_t ent) {   // column of edge k of row i
            constexpr int i = decltype(ic)::value, k = decltype(kc)::value, j = P::COL[P::RS[i] + k];
            lds_T& acc = at((uint32_t)(j * kFrColB) + ent);
            if constexpr (kFrPlan<BG>.first_row[j] == i) acc = T(0) + r;
            else __hip_atomic_fetch_add(&acc, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        T S = T(0);
        // the core LLRs of the LQ update, loaded now so phase B hides their latency
        T lf[KH];
        if (active) {
#pragma unroll
            for (int jj = 0; jj < KH; ++jj) {
                const int j = jcol(jj);
                lf[jj] = ldg(lrow, (j < pc ? 0 : j - pc) * Z + sv);
            }
            // hand-offs: the other column's message of this half's rows with both columns
            per_half([&](auto hc) {
                constexpr int H = decltype(hc)::value;
                sfor<0, MB>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    if constexpr (kFrPlan<BG>.ho[i] >= 0 && kFrPlan<BG>.owner[i] == H) {
                        if (rdead(i)) return;   // its messages are +-0: nothing to hand over
                        constexpr int k = kFrPlan<BG>.kc[1 - H][i];
                        T a, b;
                        uint32_t u, idx;
                        get_state(ic, a, b, u, idx);
                        at((uint32_t)kFrPlan<BG>.hb(kFrPlan<BG>.ho[i]) + rot(fr_cof<BG>(i, k))) =
                            msg(a, b, u, idx, std::integral_constant<int, k>{});
                    }
                });
            });
        }
        sfor<0, kFrPlan<BG>.ng>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            constexpr uint64_t gx = fr_group_xmask<BG>(g);
            const bool gdead = DEAD && gx != 0 && (live_x & gx) == 0;   // adds nothing: no barrier
            if (active && !gdead) {
                per_half([&](auto hc) {
                    constexpr int H = decltype(hc)::value;
                    sfor<kFrPlan<BG>.gstart[g], kFrPlan<BG>.gstart[g + 1]>([&](auto ic) {
                        constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = kFrPlan<BG>.deg(i);
                        if (rdead(i)) return;   // +-0 messages: no add changes a sum
                        if constexpr (kFrPlan<BG>.lds[i]) {
                            // both halves: column H's message and this half's share of the edges of
                            // columns >= 2, from the state at check node (s - Pf) mod Zc, Pf = V(i, H)
                            constexpr int Pf = fr_pf<BG>(i, H);
                            T a, b;
                            uint32_t u, idx;
                            lds_get(ic, rot((Z - Pf) % Z), a, b, u, idx);
                            sfor<0, d>([&](auto kc) {
                                constexpr int k = decltype(kc)::value, j = P::COL[e0 + k];
                                if constexpr (j == H) {
                                    S = S + xsign_v(pick(idx == (uint32_t)k, b, a), u, mv);
                                } else if constexpr (fr_item<BG>(H, i, k)) {
                                    add_to(ic, kc, xsign_v(pick(idx == (uint32_t)k, b, a), u, mv),
                                           rot((fr_sft<BG>(i, k) - Pf + Z) % Z));
                                }
                                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // u <<= 1
                            });
                        } else if constexpr (kFrPlan<BG>.owner[i] == H) {
                            // this half's VGPR row in frame H: column H's entry is this thread's own
                            T a, b;
                            uint32_t u, idx;
                            get_state(ic, a, b, u, idx);
                            sfor<0, d>([&](auto kc) {
                                constexpr int k = decltype(kc)::value, j = P::COL[e0 + k];
                                if constexpr (j == H) {
                                    S = S + xsign_v(pick(idx == (uint32_t)k, b, a), u, mv);
                                } else if constexpr (j >= 2 && j < KC) {
                                    add_to(ic, kc, xsign_v(pick(idx == (uint32_t)k, b, a), u, mv), rot(fr_cof<BG>(i, k)));
                                }
                                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));
                            });
                        } else if constexpr (kFrPlan<BG>.ho[i] >= 0 && kFrPlan<BG>.kc[H][i] >= 0) {
                            S = S + at((uint32_t)kFrPlan<BG>.hb(kFrPlan<BG>.ho[i]) + sb);   // the owner's hand-off
                        }
                    });
                });
            }
            if (!gdead) lds_barrier();
        });
        // ---- LQ = LLRin + sum (:126) for the own entries
        if (active) {
#pragma unroll
            for (int jj = 0; jj < KH; ++jj) {
                const int j = jcol(jj);
                lds_T& x = at((uint32_t)(j * kFrColB) + sb);
                x = (j < pc ? T(0) : lf[jj]) + (jj == 0 ? S : x);   // punctured columns: LLR 0 (:43)
            }
        }
        if (t == 0) *flagA = 0;   // read before the phase-B barriers
        if (!block_any(active)) break;
    }

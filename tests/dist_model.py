"""CPU model of the partitioned wave's exchange protocol (stl.fusion_amd/csrc/part.hip), run over a
real torch.distributed process group (gloo) — test infrastructure for the N>1 path, which the GPU
engine runs over RCCL. Same decomposition as part.hip:

- rank p owns slots [p*B, p*B + n_local), B = ceil(N / world): their node states and `_usedBy`
  rows (entries keep GLOBAL dependant ids); every rank holds a replica of all N versions;
- push level: expand the owned frontier; owned targets are visited locally; a remote target whose
  tag matches its replicated version is forwarded once per wave (per-wave "sent" bitmap: only a
  node's first visit in a wave can change it, Computed.cs:164-191), counts + payload exchanged
  (ncclAllGather + ncclSend/Recv on the GPU; all_gather here), owners apply them;
- pull level: the frontier bitmap is all-gathered and every rank pulls its own unvisited slots
  over their dependency lists (global parent ids), stopping at the first parent in the frontier;
- {frontier size, frontier edges} of the next level decide termination and the push/pull choice
  (Beamer's alpha and beta rules, as the engine's run_part_wave): after a pull level by one
  all_reduce(sum); after a push level from the counts all-gather, which also carries every rank's
  local next {F, T} — F + forwarded targets bounds the next frontier, T scales by local edges per
  winner — except when every winner is remote, where the all_reduce decides (exact termination).

Visits follow SURVEY.md §8(a) R0 (Computed.cs:162-230): Invalidated -> no-op; Computing -> flag
InvalidateOnSetOutput; Consistent without delay -> Invalidated + expand; Consistent with delay ->
InvalidationDelayStarted. Roots: the slot's current node, Invalidate(immediately).
"""
import numpy as np
import torch
import torch.distributed as dist

COMPUTING, CONSISTENT, INVALIDATED = 0, 1, 2
F_IOSO, F_DS, F_HD = 4, 8, 16


class RankModel:
    def __init__(self, rank, world, n, versions, flags, src, dst, tags):
        self.rank, self.world, self.n = rank, world, n
        self.B = -(-n // world)
        self.lo = rank * self.B
        self.hi = min(n, self.lo + self.B)
        self.ver_all = versions.astype(np.uint64)           # replicated, immutable during a wave
        self.flags = flags[self.lo:self.hi].astype(np.uint32).copy()
        self.ver = versions[self.lo:self.hi].astype(np.uint64).copy()
        mine = (src >= self.lo) & (src < self.hi)
        s, d, t = src[mine], dst[mine], tags[mine]
        # set semantics of `_usedBy` (HashSetSlim3): duplicate (dst, tag) entries collapse
        key = np.unique(np.stack([s.astype(np.uint64), d.astype(np.uint64), t], 1), axis=0)
        self.rows = {}
        for a, b, c in key:
            self.rows.setdefault(int(a), []).append((int(b), int(c)))
        # dependency lists for pull: owned dependant d -> global parents whose row holds (d, ver[d])
        own_d = (dst >= self.lo) & (dst < self.hi)
        self.deps = {}
        for a, b, c in zip(src[own_d], dst[own_d], tags[own_d]):
            if c == versions[b]:
                self.deps.setdefault(int(b), set()).add(int(a))
        self.sent = np.zeros(n, bool)
        self.inv = []

    def owner(self, slot):
        return slot // self.B

    def _visit(self, slot, immediately=False):
        """First visit of an owned node; returns True if it was invalidated (expands)."""
        i = slot - self.lo
        f = int(self.flags[i])
        if self.ver[i] == 0:
            return False
        st = f & 3
        if st == INVALIDATED:
            return False
        if st == COMPUTING:
            f |= F_IOSO
            if immediately:
                f |= F_DS
            self.flags[i] = f
            return False
        if (f & F_HD) and not immediately:
            self.flags[i] = f | F_DS
            return False
        self.flags[i] = INVALIDATED | (f & F_HD)   # canonical flags of an Invalidated node
        self.inv.append(slot)
        return True

    def _matches(self, slot, tag):
        return self.ver_all[slot] == tag   # replicated versions; the owner checks the state

    def wave(self, roots, immediately=None, direction="push", alpha=14, beta=24):
        self.sent[:] = False
        visited = set()
        front = []
        for k, r in enumerate(roots):
            r = int(r)
            if self.lo <= r < self.hi and r not in visited:
                visited.add(r)
                imm = bool(immediately[k]) if immediately is not None else False
                if self._visit(r, imm):
                    front.append(r)
        e_total = torch.tensor([sum(len(v) for v in self.rows.values())], dtype=torch.int64)
        dist.all_reduce(e_total)
        levels = 0
        last_pull = False
        known = None   # {frontier, its edges} from the last push level's counts all-gather
        while True:
            # termination and Beamer's rules — pull when the edges exceed E / alpha, keep pulling
            # after a pull while the frontier holds more than N / beta nodes
            if known is None:
                ft = torch.tensor([len(front), sum(len(self.rows.get(u, ())) for u in front)], dtype=torch.int64)
                dist.all_reduce(ft)
                n_front, edges = int(ft[0]), int(ft[1])
            else:
                (n_front, edges), known = known, None
            if n_front == 0:
                break
            pull = direction == "pull" or (direction == "auto" and (edges > int(e_total) // alpha or
                                                                    (last_pull and n_front > self.n // beta)))
            last_pull = pull
            nxt = []
            if pull:
                bm = np.zeros(self.n, bool)
                bm[np.asarray(front, np.int64)] = True
                parts = [torch.zeros(self.n, dtype=torch.bool) for _ in range(self.world)]
                dist.all_gather(parts, torch.from_numpy(bm))   # frontier bitmap all-gather
                gfront = np.logical_or.reduce([p.numpy() for p in parts])
                for d, ps in self.deps.items():
                    if d in visited:
                        continue
                    if any(gfront[p] for p in ps):
                        visited.add(d)
                        if self._visit(d):
                            nxt.append(d)
            else:
                out = [[] for _ in range(self.world)]
                for u in front:
                    for d, t in self.rows.get(u, ()):
                        if not self._matches(d, t):
                            continue
                        q = self.owner(d)
                        if q == self.rank:
                            if d not in visited:
                                visited.add(d)
                                if self._visit(d):
                                    nxt.append(d)
                        elif not self.sent[d]:
                            self.sent[d] = True
                            out[q].append(d)
                # counts (+ local next F, T) then payload (ncclAllGather + ncclSend/ncclRecv on the GPU)
                f_loc, t_loc = len(nxt), sum(len(self.rows.get(u, ())) for u in nxt)
                cnt = torch.tensor([len(o) for o in out] + [f_loc, t_loc], dtype=torch.int64)
                all_cnt = [torch.zeros(self.world + 2, dtype=torch.int64) for _ in range(self.world)]
                dist.all_gather(all_cnt, cnt)
                f_sum = sum(int(c[self.world]) for c in all_cnt)
                t_sum = sum(int(c[self.world + 1]) for c in all_cnt)
                sent = sum(int(c[:self.world].sum()) for c in all_cnt)
                if f_sum or not sent:
                    n_est = f_sum + sent
                    t_est = int(t_sum * n_est / f_sum) if f_sum else int(sent * int(e_total) / self.n)
                    known = (n_est, max(t_est, 1) if sent else t_est)
                width = max(1, int(max(int(c[:self.world].max()) for c in all_cnt)))
                pay = torch.full((self.world, width), -1, dtype=torch.int64)
                for q, o in enumerate(out):
                    if o:
                        pay[q, :len(o)] = torch.tensor(o, dtype=torch.int64)
                all_pay = [torch.zeros_like(pay) for _ in range(self.world)]
                dist.all_gather(all_pay, pay)
                for r in range(self.world):
                    c = int(all_cnt[r][self.rank])
                    for d in all_pay[r][self.rank, :c].tolist():
                        if d not in visited:
                            visited.add(d)
                            if self._visit(d):
                                nxt.append(d)
            front = nxt
            levels += 1
        return levels

    def gather_results(self):
        """Union of the invalidated sets and the owners' final flags, on every rank."""
        inv = [None] * self.world
        dist.all_gather_object(inv, sorted(self.inv))
        fl = [None] * self.world
        dist.all_gather_object(fl, self.flags.tolist())
        return sorted(x for part in inv for x in part), np.concatenate([np.asarray(f, np.uint32) for f in fl])


# ---- the registry's mutations on a partition (part_* in stl.fusion_amd/csrc/graph.hip) -----------
# Every rank makes the same call with the same global arrays; each applies its own slots. A displaced
# node leaves the slot (its handle is local and unreachable through slot ids), so the model drops it.

def _own(m, s):
    return m.lo <= s < m.hi


def begin_compute(m, slots, versions, has_delay, direction="auto"):
    """ComputedRegistry.Register with displacement (ComputedRegistry.cs:83-97): the owners' current
    Consistent undelayed nodes are the displacement cascade's roots (one partitioned wave); then every
    rank records the new versions in its replica and the owners install Computing nodes with empty
    `_usedBy` / `_used`."""
    roots = []
    det = torch.zeros(len(slots), dtype=torch.int64)
    for k, s in enumerate(slots):
        s = int(s)
        if _own(m, s):
            i = s - m.lo
            f = int(m.flags[i])
            if m.ver[i] != 0 and (f & 3) == CONSISTENT and not (f & F_HD):
                roots.append(s)
            elif m.ver[i] != 0 and (f & 3) != INVALIDATED:
                det[k] = 1      # displaced while current: detached, out of every slot-addressed path
    dist.all_reduce(det)
    gone = {int(s) for k, s in enumerate(slots) if det[k]}
    for d in m.deps:
        m.deps[d] -= gone
    m.wave(roots, direction=direction, alpha=6)
    for s, v, h in zip(slots, versions, has_delay):
        s = int(s)
        m.ver_all[s] = v
        if _own(m, s):
            i = s - m.lo
            m.ver[i] = v
            m.flags[i] = COMPUTING | (F_HD if h else 0)
            m.rows[s] = []
            m.deps.pop(s, None)


def add_used(m, dep, used):
    """AddUsed / AddUsedBy (Computed.cs:347-385) for pairs whose ends may live on different ranks:
    the dependant's owner says whether it is Computing (all-reduce), the used node's owner applies the
    rules and appends (dependant, version), the codes are all-reduced, the dependant's owner flags
    InvalidateOnSetOutput or records the dependency. Returns the FGI_USED_* codes (every rank)."""
    n = len(dep)
    comp = torch.zeros(n, dtype=torch.int64)
    for k in range(n):
        d = int(dep[k])
        if _own(m, d):
            i = d - m.lo
            comp[k] = int(m.ver[i] != 0 and (int(m.flags[i]) & 3) == COMPUTING)
    dist.all_reduce(comp)
    res = torch.zeros(n, dtype=torch.int64)
    for k in range(n):
        d, u = int(dep[k]), int(used[k])
        if not _own(m, u):
            continue
        j = u - m.lo
        st = int(m.flags[j]) & 3
        if not comp[k]:
            code = 1                                   # dropped
        elif m.ver[j] == 0 or st == INVALIDATED:
            code = 2                                   # invalidated
        elif st == COMPUTING:
            code = 3                                   # wrong state
        else:
            code = 0
            e = (d, int(m.ver_all[d]))
            row = m.rows.setdefault(u, [])
            if e not in row:
                row.append(e)
        res[k] = code + 1
    dist.all_reduce(res)
    codes = (res - 1).numpy()
    for k in range(n):
        d, u = int(dep[k]), int(used[k])
        if _own(m, d):
            if codes[k] == 2:
                m.flags[d - m.lo] |= F_IOSO
            elif codes[k] == 0:
                m.deps.setdefault(d, set()).add(u)
    return codes


def set_output(m, slots, direction="auto"):
    """TrySetOutput (Computed.cs:141-160): the owners' Computing nodes become Consistent; those flagged
    InvalidateOnSetOutput are the roots of one partitioned wave. Returns how many were set."""
    setf = torch.zeros(len(slots), dtype=torch.int64)
    roots = []
    for k, s in enumerate(slots):
        s = int(s)
        if _own(m, s):
            i = s - m.lo
            f = int(m.flags[i])
            if m.ver[i] != 0 and (f & 3) == COMPUTING:
                setf[k] = 1
                m.flags[i] = CONSISTENT | (f & (F_HD | F_DS))
                if f & F_IOSO:
                    roots.append(s)
    m.wave(roots, direction=direction, alpha=6)
    dist.all_reduce(setf)
    return int(setf.sum())


def prune(m):
    """PruneUsedBy (Computed.cs:400-419) on the owners' Consistent nodes: an entry stays iff its
    dependant is registered (current, not Invalidated) at the entry's version; "current" comes from an
    all-gather of the owners' states (the engine's current-node bitmap), the version from the replica.
    Returns the entries left on this rank."""
    cur = np.zeros(m.n, bool)
    mine = np.zeros(m.hi - m.lo, bool)
    mine[:] = (m.ver != 0) & ((m.flags & 3) != INVALIDATED)
    cur[m.lo:m.hi] = mine
    parts = [torch.zeros(m.n, dtype=torch.bool) for _ in range(m.world)]
    dist.all_gather(parts, torch.from_numpy(cur))
    cur = np.logical_or.reduce([p.numpy() for p in parts])
    left = 0
    for u, row in m.rows.items():
        i = u - m.lo
        if m.ver[i] == 0 or (int(m.flags[i]) & 3) != CONSISTENT:
            continue
        m.rows[u] = [(d, t) for d, t in row if cur[d] and m.ver_all[d] == t]
        left += len(m.rows[u])
    return left


def live_rows(m):
    """(used, dependant, tag) of the `_usedBy` rows of this rank's registered nodes."""
    out = []
    for u, row in m.rows.items():
        i = u - m.lo
        if m.ver[i] == 0 or (int(m.flags[i]) & 3) == INVALIDATED:
            continue
        out += [(u, d, t) for d, t in row]
    return out


# ---- planned waves (run_part_planned in stl.fusion_amd/csrc/wave.hip) ----------------------------
# A wave follows a plan (per-level push/pull, learnt from an earlier wave) with fixed-size exchanges:
# a pull level all-gathers the whole invalidated bitmap; a push level sends each peer a bucket of C
# words (a count, then at most C - 1 ids) and keeps the ids that did not fit for the next push level;
# after the plan's levels, push levels are appended while any rank still holds ids to send or has a
# frontier. One closing all-reduce decides that (the engine's one host synchronisation per round).

def planned_wave(m, roots, plan, C, immediately=None):
    """Returns (levels run, rounds)."""
    m.sent[:] = False
    visited = set()
    front = []
    for k, r in enumerate(roots):
        r = int(r)
        if m.lo <= r < m.hi and r not in visited:
            visited.add(r)
            imm = bool(immediately[k]) if immediately is not None else False
            if m._visit(r, imm):
                front.append(r)
    pending = [[] for _ in range(m.world)]   # ids waiting for a bucket, per owner
    levels = rounds = 0
    seq = list(plan)
    while True:
        rounds += 1
        for pull in seq:
            nxt = []
            if pull:
                bm = np.zeros(m.n, bool)
                # the whole invalidated bitmap: every invalidated owned slot so far, as the engine's
                # inv_bm (a pull probes parents invalidated at any earlier level)
                for x in m.inv:
                    bm[x] = True
                parts = [torch.zeros(m.n, dtype=torch.bool) for _ in range(m.world)]
                dist.all_gather(parts, torch.from_numpy(bm))
                g = np.logical_or.reduce([p.numpy() for p in parts])
                for d, ps in m.deps.items():
                    if d in visited:
                        continue
                    if any(g[p] for p in ps):
                        visited.add(d)
                        if m._visit(d):
                            nxt.append(d)
            else:
                for u in front:
                    for d, t in m.rows.get(u, ()):
                        if not m._matches(d, t):
                            continue
                        q = m.owner(d)
                        if q == m.rank:
                            if d not in visited:
                                visited.add(d)
                                if m._visit(d):
                                    nxt.append(d)
                        elif not m.sent[d]:
                            m.sent[d] = True
                            pending[q].append(d)
                # fixed-size buckets: a count word, then up to C - 1 ids per peer
                send = torch.zeros((m.world, C), dtype=torch.int64)
                for q in range(m.world):
                    if q == m.rank:
                        continue
                    take, pending[q] = pending[q][:C - 1], pending[q][C - 1:]
                    send[q, 0] = len(take)
                    if take:
                        send[q, 1:1 + len(take)] = torch.tensor(take, dtype=torch.int64)
                recv = torch.zeros((m.world, C), dtype=torch.int64)
                dist.all_to_all_single(recv, send)
                for q in range(m.world):
                    for d in recv[q, 1:1 + int(recv[q, 0])].tolist():
                        if d not in visited:
                            visited.add(d)
                            if m._visit(d):
                                nxt.append(d)
            front = nxt
            levels += 1
        left = torch.tensor([len(front), sum(len(p) for p in pending)], dtype=torch.int64)
        dist.all_reduce(left)
        if int(left[0]) == 0 and int(left[1]) == 0:
            return levels, rounds
        seq = [0] * 4   # more push levels while ids wait or a frontier is left

"""Progress checker for the dataflow launches' claim protocols.

A dataflow launch (the natural-SSOR units and chains of ssor_natural.hip, the ILU(0) units of
linalg.hip k_ilu0_flow) is a DAG of units, every dependency earlier in a global unit order, worked
by the workgroups (or waves) of one grid.  A worker claims a unit and then spins inside it until
its predecessors are final; it never gives a claimed unit back.  Only R of the grid's G workers are
resident at once: the dispatcher starts workers in index order and starts worker R + i only after
some resident worker has exited.  A launch can hang iff some reachable state has every resident
worker spinning on a unit with an unfinished predecessor that no running worker will complete.

simulate() plays the protocol against an adversary that makes every free worker claim before any
unit completes (claims are what commit a worker) and then completes one claimable unit at a time,
in an order drawn from a seeded random stream (several seeds per check).  It returns the first
deadlocked state found, or None.  Protocols (Claimer subclasses):
  Static(G)          worker w takes units w, w + G, w + 2G, ... in order (k_ssor_nat_flow / _pipe,
                     the resident-grid ILU(0) flow): deadlock-free iff R >= G (the earliest
                     unfinished unit's worker has finished its own earlier units);
  Ticket()           one global counter, units in the global order (the ticketed ILU(0) flow,
                     PNP_OPT_ILU_FLOW = 2): deadlock-free for every R >= 1;
  Groups(seqs)       worker g walks the fixed sequence seqs[g] (k_ssor_nat_chain's chain groups):
                     deadlock-free iff every group is resident and each sequence follows the
                     global order;
  Queues(Q, home)    round 4's removed form: Q ticket queues (unit u in queue home(u)), worker w
                     reads queue w % Q and, once that queue has handed out all its tickets, takes
                     tickets from the other queues in turn -- claims then leave the global order,
                     and a queue whose home workers are not all resident loses its only readers
                     while every resident worker spins on a stolen unit behind it;
  Queues(..., steal_ready=True)  the fix round 4's verdict proposed: a foreign ticket is taken only
                     if every predecessor of its unit is already claimed -- NOT enough: a resident
                     worker still spins on a unit of its OWN queue whose predecessor sits in a
                     queue with no resident home worker;
  Queues(..., ready_all=True)  every claim (own queue or foreign) only of a queue head whose
                     predecessors are all claimed, else the worker polls again holding nothing:
                     deadlock-free for every R >= 1 (the smallest unclaimed unit is a queue head
                     whose predecessors, all smaller, are claimed; the smallest unfinished claimed
                     unit's predecessors are finished).
usage: python tools/claim_check.py   (runs the demonstration cases; tests/test_claim_check.py)"""
import random


def probe_arrivals(G, R, hold=True):
    """The co-residency probe of ssor_natural.hip (nat_probe): the grid's G workers each check in
    and wait, bounded, until all G have; the dispatcher starts worker R + i only after a resident
    worker exits.  Returns the largest arrival count any waiting worker can observe before its
    wait ends (hold: workers hold their slot while they wait, as the probe's wave does).  The
    probe passes iff that count reaches G; otherwise every waiting worker times out, exits, and
    the launch drains with the flag set -- the context then keeps the level launches."""
    if not hold:
        return G
    return min(G, R)


class Claimer:
    def reset(self, n, deps):
        self.n, self.deps = n, deps

    def claim(self, w, claimed):
        raise NotImplementedError


class Static(Claimer):
    def __init__(self, G):
        self.G = G

    def reset(self, n, deps):
        super().reset(n, deps)
        self.nxt = {}

    def claim(self, w, claimed):
        u = self.nxt.get(w, w)
        if u >= self.n:
            return None
        self.nxt[w] = u + self.G
        return u


class Ticket(Claimer):
    def reset(self, n, deps):
        super().reset(n, deps)
        self.t = 0

    def claim(self, w, claimed):
        if self.t >= self.n:
            return None
        self.t += 1
        return self.t - 1


class Groups(Claimer):
    def __init__(self, seqs):
        self.seqs = seqs

    def reset(self, n, deps):
        super().reset(n, deps)
        self.pos = [0] * len(self.seqs)

    def claim(self, w, claimed):
        if w >= len(self.seqs) or self.pos[w] >= len(self.seqs[w]):
            return None
        self.pos[w] += 1
        return self.seqs[w][self.pos[w] - 1]


WAIT = -1  # a free worker that found nothing it may claim yet (it polls again, holding nothing)


class Queues(Claimer):
    def __init__(self, Q, home, steal_ready=False, ready_all=False):
        self.Q, self.home, self.steal_ready, self.ready_all = Q, home, steal_ready, ready_all

    def reset(self, n, deps):
        super().reset(n, deps)
        self.q = [[u for u in range(n) if self.home(u) == k] for k in range(self.Q)]
        self.t = [0] * self.Q

    def claim(self, w, claimed):
        q0 = w % self.Q
        left = False
        for k in range(self.Q):
            q = (q0 + k) % self.Q
            if self.t[q] >= len(self.q[q]):
                continue
            left = True
            u = self.q[q][self.t[q]]
            if (self.ready_all or (k > 0 and self.steal_ready)) and \
                    not all(claimed[p] for p in self.deps[u]):
                continue  # take only a unit whose predecessors are all claimed
            self.t[q] += 1
            return u
        return WAIT if left else None


def simulate(n, deps, proto, G, R, seed=0):
    """Returns None if the launch drains, else a dict describing the deadlocked state."""
    rng = random.Random(seed)
    proto.reset(n, deps)
    claimed, done = [False] * n, [False] * n
    held = {}              # resident worker -> unit it spins in (None: free)
    started = 0            # workers started so far (in index order)
    exited = set()
    ndone = 0
    while True:
        while len(held) < R and started < G:  # the dispatcher fills the free slots in order
            held[started] = None
            started += 1
        progress = True
        while progress:  # every free worker claims before anything completes
            progress = False
            for w in sorted(held):
                if held[w] is None:
                    u = proto.claim(w, claimed)
                    if u == WAIT:
                        continue
                    if u is None:
                        del held[w]
                        exited.add(w)
                        while len(held) < R and started < G:
                            held[started] = None
                            started += 1
                        progress = True
                        break
                    claimed[u] = True
                    held[w] = u
                    progress = True
        if ndone == n:
            return None
        ready = [w for w, u in held.items() if u is not None and all(done[p] for p in deps[u])]
        if not ready:
            spin = {w: u for w, u in held.items() if u is not None}
            return {"resident": len(held), "started": started, "done": ndone,
                    "spinning": {w: (u, [p for p in deps[u] if not done[p]]) for w, u in
                                 list(spin.items())[:8]},
                    "unclaimed_blockers": sorted({p for u in spin.values() for p in deps[u]
                                                  if not claimed[p]})[:8]}
        w = rng.choice(ready)
        done[held[w]] = True
        ndone += 1
        held[w] = None


def check(n, deps, proto, G, R, seeds=8):
    for s in range(seeds):
        r = simulate(n, deps, proto, G, R, s)
        if r is not None:
            return r
    return None


def layered_dag(nlev, width, fan, seed=1):
    """A level-structured DAG like the sweeps': `width` units per level, each depending on up to
    `fan` random units of the level below; units numbered level by level (the global order)."""
    rng = random.Random(seed)
    deps = []
    for L in range(nlev):
        for _ in range(width):
            if L == 0:
                deps.append([])
            else:
                lo = (L - 1) * width
                deps.append(sorted({lo + rng.randrange(width) for _ in range(fan)}))
    return len(deps), deps


def main():
    n, deps = layered_dag(12, 16, 3)
    G = 16
    print("static, R = G:", check(n, deps, Static(G), G, G))
    print("static, R = G - 1:", check(n, deps, Static(G), G, G - 1) is not None)
    print("ticket, R = 3:", check(n, deps, Ticket(), G, 3))
    home = lambda u: (u * 5) % 8  # noqa: E731
    print("8 queues, every queue resident:", check(n, deps, Queues(8, home), 16, 16))
    print("8 queues, R = 5:", check(n, deps, Queues(8, home), 16, 5) is not None)
    print("8 queues + ready steal, R = 5:", check(n, deps, Queues(8, home, True), 16, 5) is not None)
    print("8 queues + ready claims, R = 5:", check(n, deps, Queues(8, home, ready_all=True), 16, 5))
    print("8 queues + ready claims, R = 1:", check(n, deps, Queues(8, home, ready_all=True), 16, 1))


if __name__ == "__main__":
    main()

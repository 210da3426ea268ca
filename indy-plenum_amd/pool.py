"""A minimal in-process n-node pool for end-to-end measurement of the
authentication path (Alpha-Delta under a
client-request flood).  The reference pool cannot run in this image (zmq,
rocksdb, indy-crypto, libindy and Python <= 3.6 are absent), so this harness
keeps exactly the parts of the Node message flow that decide how often and where
request signatures are verified, and reduces the rest to message counting:

  client REQUEST to every node        plenum/server/node.py:1646-1743 (verify)
    -> processRequest: record, PROPAGATE to all   node.py:2093-2143,
                                                  propagator.py:165-183, 251-261
  PROPAGATE from a peer               node.py:1553-1620 (verify again),
    -> processPropagate: vote, propagate once     node.py:2183-2230
  f+1 PROPAGATE votes -> finalised, forwarded     propagator.py:200-249
  master replica 3PC: the primary batches finalised requests into a
    PRE-PREPARE, PREPARE quorum n-f-1, COMMIT quorum n-f, ordered in
    ppSeqNo order                                 plenum/server/replica.py
  node-to-node messages are JSON-encoded and flushed once per prod per peer
    as one batch                                  node.py:1049 flushOutBoxes

Not modelled (out of scope): view change, checkpoints,
catch-up, BLS multi-signatures, ledgers/state execution, client replies.

Fault injection as in the reference's signing test (plenum/test/signing/
test_signing.py:30-77 with malicious_behaviors_node.py:31-44 changesRequest):
a node named in Pool(..., alters_propagates={...}) puts a random "amount" into
the operation of every request it PROPAGATEs, so the client's signature no
longer matches; the other nodes' authentication of those PROPAGATEs fails with
InsufficientCorrectSignatures(0, 1), they record the sender as suspicious
(Node.reportSuspiciousNode) and do not count its vote.

Request latency (what the reference's Monitor acts on, plenum/server/monitor.py:
300-330 requestOrdered, :418-460 LAMBDA / OMEGA checks) is recorded per request
and node: from forwarding (f+1 PROPAGATE votes, propagator.py:236-249, where
the Monitor starts its clock) to ordering ("monitor"), from the prod that read
the request off the node's inbox to ordering ("receipt"), and from the client's
submission to ordering ("submit").  run_paced() offers the requests at a fixed
rate instead of all at once, so latency is measured below saturation.

Each node authenticates through a ReqAuthenticator; `batched=True` routes a
prod's client REQUESTs and PROPAGATEs through ONE authenticate_batch call
(node_integration.authenticate_prod), `batched=False` is the reference's
one-message-at-a-time verifySignature.  Request keys are Request.getDigest
(request.py:71-72) values computed by `digest_fn`.

`overlap=True` (batched only) submits a prod's authentication batch without
waiting (ReqAuthenticator.authenticate_batch_submit: host prep now, one queued
device call that also hashes the request digests) and handles its verdicts
later, so the GPU round trip of one node's batch runs while the node does its
Python work: with handover="early" (default) at the end of the same prod if
the GPU is done by then (PendingProd.ready, a non-blocking edv_query_async),
else at the node's next prod; with handover="next" always at the next prod.
Each message is still handled exactly once with its own verdict, in arrival
order.
"""
import gc
import hashlib
import json
import random
import time
from collections import deque

from .node_integration import DEFAULT_LISTENER_QUOTA, PendingProd, authenticate_prod, failed
from .signing_serializer import serialize_msg_for_signing
from .digest import signing_state

NAMES = ("Alpha", "Beta", "Gamma", "Delta", "Epsilon", "Zeta", "Eta", "Theta")


def cpu_digests(reqs):
    """Request.getDigest on the host (hashlib), one request at a time."""
    return [hashlib.sha256(serialize_msg_for_signing(signing_state(r))).hexdigest() for r in reqs]


def _as_outcome(r):
    """authenticate_batch's per-request result as authenticate_prod's outcome:
    the identifier set, or the exception instance verifySignature would raise."""
    return r


class _ReqState:
    __slots__ = ("votes", "propagated", "forwarded")

    def __init__(self):
        self.votes = set()
        self.propagated = False
        self.forwarded = False


class _GcClock:
    """Seconds the cyclic GC ran, in total and while a node was inside its
    authentication window (the GC runs when the process's allocation count
    crosses a threshold, so a collection lands in whichever code allocates
    next, and pays for every object the node made, not only the ones it made
    there)."""

    def __init__(self):
        self.total_s = self.in_auth_s = 0.0
        self.auth_depth = 0
        self._t = None

    def __call__(self, phase, _info):
        if phase == "start":
            self._t = time.perf_counter()
        elif self._t is not None:
            d = time.perf_counter() - self._t
            self.total_s += d
            if self.auth_depth:
                self.in_auth_s += d
            self._t = None


class _AuthWindow:
    """Adds the time spent inside it to node.auth_s."""
    __slots__ = ("node", "t")

    def __init__(self, node):
        self.node = node

    def __enter__(self):
        self.node.gc_clock.auth_depth += 1
        self.t = time.perf_counter()

    def __exit__(self, *exc):
        self.node.auth_s += time.perf_counter() - self.t
        self.node.gc_clock.auth_depth -= 1


class _TimedAuth:
    """ReqAuthenticator proxy adding the time spent inside it to node.auth_s."""

    def __init__(self, auth, node):
        self._auth, self._node = auth, node

    def authenticate(self, req):
        with _AuthWindow(self._node):
            return self._auth.authenticate(req)

    def authenticate_batch(self, reqs):
        with _AuthWindow(self._node):
            return self._auth.authenticate_batch(reqs)

    def authenticate_batch_submit(self, reqs, digests=False):
        # timed by the caller (PoolNode.prod), together with the hand-over
        return self._auth.authenticate_batch_submit(reqs, digests=digests)


class PoolNode:
    def __init__(self, name, peers, authenticator, f, batched=True, digest_fn=cpu_digests,
                 client_quota=DEFAULT_LISTENER_QUOTA, node_quota=DEFAULT_LISTENER_QUOTA, max_batch=1000,
                 overlap=False, handover="early", alters_propagates=False):
        self.name, self.peers, self.f = name, list(peers), f
        # fault injection: this node's PROPAGATEs carry an altered request
        # (malicious_behaviors_node.py:31-44 changesRequest)
        self.alters_propagates = alters_propagates
        self._rng = random.Random(name)
        self.overlap = overlap and batched
        if handover not in ("early", "next"):
            raise ValueError("handover must be 'early' or 'next'")
        # overlap mode: "early" hands a prod's batch over at the end of the same
        # prod when the GPU is already done (PendingProd.ready), else at the next
        # prod; "next" always at the next prod
        self.early = handover == "early"
        self.early_handovers = 0
        self._pending = None          # PendingProd not yet handed over (overlap mode)
        self.auth = _TimedAuth(authenticator, self)
        self.n = len(self.peers) + 1
        self.batched, self.digest_fn = batched, digest_fn
        self.client_quota, self.node_quota, self.max_batch = client_quota, node_quota, max_batch
        self.client_inbox = deque()   # JSON text of client REQUESTs
        self.node_inbox = deque()     # (frm, JSON text of one flushed batch)
        self.outbox = {p: [] for p in self.peers}
        self.requests = {}            # key -> _ReqState
        self.ordered_keys = set()
        self.finalised = deque()      # finalised keys not yet in a PRE-PREPARE (primary)
        self.finalised_set = set()
        self.is_primary = False
        # master replica state
        self.pp = {}                  # ppSeqNo -> list of keys
        self.pp_waiting = []          # ppSeqNos received but not all requests finalised yet
        self.prepares = {}            # ppSeqNo -> set of senders
        self.commits = {}             # ppSeqNo -> set of senders
        self.sent_prepare, self.sent_commit = set(), set()
        self.last_pp = 0
        self.last_ordered = 0
        # counters
        self.ordered = 0
        self.nacks = 0
        self.bad_propagates = 0
        self.suspicions = []          # (sender, reason) per PROPAGATE that failed authentication
        self.verifies = 0
        self.auth_calls = 0
        self.busy_s = 0.0
        self.auth_s = 0.0             # time inside request authentication and request digests
        self.gc_clock = _GcClock()    # replaced by the pool's shared clock
        # latency bookkeeping (perf_counter seconds)
        self._pool = None
        self._t_read = 0.0            # start of the prod that read the messages being handled
        self.t_recv, self.t_fwd, self.key_rid = {}, {}, {}
        self.lat = {"monitor": [], "receipt": [], "submit": []}

    # ------------------------------------------------------------------ I/O
    def send_all(self, msg):
        for p in self.peers:
            self.outbox[p].append(msg)

    def flush(self, pool):
        for p, msgs in self.outbox.items():
            if msgs:
                pool.nodes[p].node_inbox.append((self.name, json.dumps(msgs)))
                self.outbox[p] = []

    # ------------------------------------------------------------------ prod
    def prod(self, pool):
        t0 = time.perf_counter()
        self._pool = pool
        props, three_pc = [], []
        for _ in range(min(self.node_quota, len(self.node_inbox))):
            frm, blob = self.node_inbox.popleft()
            for m in json.loads(blob):
                (props if m["op"] == "PROPAGATE" else three_pc).append((m, frm))
        clients = [(json.loads(self.client_inbox.popleft()), "client")
                   for _ in range(min(self.client_quota, len(self.client_inbox)))]
        if self.overlap:
            pend, self._pending = self._pending, None
            if props or clients:
                self.verifies += len(props) + len(clients)
                self.auth_calls += 1
                with _AuthWindow(self):
                    self._pending = PendingProd(self.auth, clients, props, digests=True)
                self._pending.t_read = t0
            if pend is not None:
                self._finish(pend)
        elif props or clients:
            with _AuthWindow(self):
                keys = self.digest_fn([m["request"] for m, _ in props] + [m for m, _ in clients])
            self._keys = iter(keys)
            self.verifies += len(props) + len(clients)
            self.auth_calls += 1 if self.batched else len(props) + len(clients)
            self._t_read = t0
            authenticate_prod(self.auth, clients, props, self._on_client, self._on_propagate, self.batched)
        n_work = len(props) + len(clients) + len(three_pc) + (self._pending is not None)
        for m, frm in three_pc:
            getattr(self, "_on_" + m["op"])(m, frm)
        if self.early and self._pending is not None:
            with _AuthWindow(self):
                done = self._pending.ready()
            if done:  # this prod's batch is verified already: hand it over now
                pend, self._pending = self._pending, None
                self.early_handovers += 1
                self._finish(pend)
        self._service_replica()
        self.flush(pool)
        self.busy_s += time.perf_counter() - t0
        return n_work

    # overlap mode: the previous prod's verdicts and digests, handed over now
    def _finish(self, pend):
        # waits only for what did not overlap, and builds the verdict lists
        with _AuthWindow(self):
            keys = pend.digests(self.digest_fn)
        self._keys = iter(keys)
        self._t_read = pend.t_read
        pend.finish(self._on_client, self._on_propagate)

    # ------------------------------------------------------- requests
    def _on_client(self, req, frm, outcome):
        key = next(self._keys)
        if failed(outcome):
            self.nacks += 1           # handleInvalidClientMsg: REQNACK to the client
            return
        if key in self.ordered_keys:
            return                    # already ordered: the reference replies from the ledger
        self._seen(key, req)
        self._record_and_propagate(key, req, frm)

    def _on_propagate(self, msg, frm, outcome):
        key = next(self._keys)
        ex = failed(outcome)
        if ex is not None:
            self.bad_propagates += 1  # SuspiciousNode
            self.suspicions.append((frm, getattr(ex, "reason", str(ex))))   # Node.reportSuspiciousNode
            return
        if key in self.ordered_keys:
            return
        st = self.requests.get(key)
        if st is None:
            st = self.requests[key] = _ReqState()
        st.votes.add(frm)
        self._seen(key, msg["request"])
        self._record_and_propagate(key, msg["request"], msg.get("senderClient"))

    def _seen(self, key, req):
        if key not in self.t_recv:
            self.t_recv[key] = self._t_read
            self.key_rid[key] = req.get("reqId")

    def _record_and_propagate(self, key, req, client):
        st = self.requests.get(key)
        if st is None:
            st = self.requests[key] = _ReqState()
        if not st.propagated:
            st.propagated = True
            st.votes.add(self.name)
            if self.alters_propagates:  # changesRequest: the signature no longer matches
                req = dict(req, operation=dict(req.get("operation") or {}, amount=self._rng.randint(10, 100000)))
            self.send_all({"op": "PROPAGATE", "request": req, "senderClient": client})
        if not st.forwarded and len(st.votes) >= self.f + 1:   # Quorums.propagate = f + 1
            st.forwarded = True
            self.t_fwd[key] = time.perf_counter()   # Monitor.requestUnOrdered (propagator.py:248)
            self.finalised_set.add(key)
            if self.is_primary:
                self.finalised.append(key)

    # ------------------------------------------------------- master replica (3PC)
    def _service_replica(self):
        if self.is_primary:
            while self.finalised:
                keys = [self.finalised.popleft() for _ in range(min(self.max_batch, len(self.finalised)))]
                self.last_pp += 1
                self.pp[self.last_pp] = keys
                self.send_all({"op": "PREPREPARE", "ppSeqNo": self.last_pp, "reqIdr": keys})
        still = []
        for s in self.pp_waiting:
            if all(k in self.finalised_set for k in self.pp[s]):
                self._send_prepare(s)
            else:
                still.append(s)
        self.pp_waiting = still
        self._try_order()

    def _on_PREPREPARE(self, m, frm):
        s = m["ppSeqNo"]
        self.pp[s] = m["reqIdr"]
        self.pp_waiting.append(s)

    def _send_prepare(self, s):
        if s not in self.sent_prepare:
            self.sent_prepare.add(s)
            self.prepares.setdefault(s, set()).add(self.name)
            self.send_all({"op": "PREPARE", "ppSeqNo": s})
            self._check_prepared(s)

    def _on_PREPARE(self, m, frm):
        s = m["ppSeqNo"]
        self.prepares.setdefault(s, set()).add(frm)
        self._check_prepared(s)

    def _check_prepared(self, s):
        # prepare quorum n - f - 1 (the primary sends none); a non-primary also needs its own PREPARE
        if s in self.sent_commit or s not in self.pp:
            return
        if not self.is_primary and s not in self.sent_prepare:
            return
        others = len(self.prepares.get(s, set()) - {self.name})
        need = self.n - self.f - 1
        if others + (0 if self.is_primary else 1) >= need:
            self.sent_commit.add(s)
            self.commits.setdefault(s, set()).add(self.name)
            self.send_all({"op": "COMMIT", "ppSeqNo": s})

    def _on_COMMIT(self, m, frm):
        self.commits.setdefault(m["ppSeqNo"], set()).add(frm)

    def _try_order(self):
        while True:
            s = self.last_ordered + 1
            if s not in self.sent_commit or len(self.commits.get(s, ())) < self.n - self.f:
                return
            keys = self.pp.pop(s)
            now = time.perf_counter()
            sub = self._pool.submit_t if self._pool is not None else {}
            for k in keys:
                if k in self.t_fwd:
                    self.lat["monitor"].append(now - self.t_fwd.pop(k))
                if k in self.t_recv:
                    self.lat["receipt"].append(now - self.t_recv.pop(k))
                rid = self.key_rid.pop(k, None)
                if rid in sub:
                    self.lat["submit"].append(now - sub[rid])
                self.ordered_keys.add(k)
                self.requests.pop(k, None)
                self.finalised_set.discard(k)
            self.ordered += len(keys)
            self.last_ordered = s
            self.prepares.pop(s, None)
            self.commits.pop(s, None)


class Pool:
    """n nodes (f = (n - 1) // 3), primary = the first; `auth_factory(name)`
    returns each node's ReqAuthenticator."""

    def __init__(self, auth_factory, n=4, batched=True, digest_fn=cpu_digests, overlap=False, alters_propagates=(),
                 **node_kw):
        names = NAMES[:n]
        f = (n - 1) // 3
        self.nodes = {nm: PoolNode(nm, [p for p in names if p != nm], auth_factory(nm), f, batched, digest_fn,
                                   overlap=overlap, alters_propagates=nm in alters_propagates, **node_kw)
                      for nm in names}
        self.nodes[names[0]].is_primary = True
        self.gc_clock = _GcClock()
        for nd in self.nodes.values():
            nd.gc_clock = self.gc_clock
        self.submit_t = {}            # reqId -> submission time

    def submit(self, reqs):
        """A client flood: every request sent to every node (as the client does)."""
        now = time.perf_counter()
        for r in reqs:
            blob = json.dumps(r)
            self.submit_t[r.get("reqId")] = now
            for node in self.nodes.values():
                node.client_inbox.append(blob)

    def run_paced(self, reqs, rate, expect=None, max_idle_s=30.0):
        """Offer `reqs` at `rate` requests/s (request i is sent at i / rate s
        after the start) while prodding every node round-robin, until `expect`
        (default: all of them) are ordered on every node; returns the
        wall-clock seconds."""
        gc.callbacks.append(self.gc_clock)
        try:
            t0 = time.perf_counter()
            sent, n = 0, len(reqs)
            target = n if expect is None else expect
            last_progress, last_min = t0, -1
            while True:
                now = time.perf_counter()
                due = min(n, int((now - t0) * rate) + 1)
                if due > sent:
                    self.submit(reqs[sent:due])
                    sent = due
                for nd in self.nodes.values():
                    nd.prod(self)
                m = min(nd.ordered for nd in self.nodes.values())
                if m >= target and sent == n:
                    break
                if m != last_min:
                    last_min, last_progress = m, now
                elif now - last_progress > max_idle_s:
                    self.drain()
                    raise RuntimeError("paced pool stalled: ordered %d of %d" % (m, target))
            self.drain()
            return time.perf_counter() - t0
        finally:
            gc.callbacks.remove(self.gc_clock)

    def run(self, expect, max_idle_rounds=50):
        """prod every node round-robin until `expect` requests are ordered on
        every node; returns the wall-clock seconds."""
        gc.callbacks.append(self.gc_clock)
        try:
            t0 = time.perf_counter()
            idle = 0
            while min(nd.ordered for nd in self.nodes.values()) < expect:
                work = sum(nd.prod(self) for nd in self.nodes.values())
                idle = 0 if work else idle + 1
                if idle > max_idle_rounds:
                    self.drain()
                    raise RuntimeError("pool stalled: ordered %s of %d" % (
                        [nd.ordered for nd in self.nodes.values()], expect))
            self.drain()
            return time.perf_counter() - t0
        finally:
            gc.callbacks.remove(self.gc_clock)

    def drain(self):
        """Overlap mode: handle every batch still in flight (its verdicts are
        applied as the node's next prod would), so no future outlives run()."""
        for nd in self.nodes.values():
            pend, nd._pending = nd._pending, None
            if pend is not None:
                nd._finish(pend)

    def close(self):
        """Hand over whatever is still in flight (the pool stays usable)."""
        self.drain()

    def stats(self, wall_s, n_reqs):
        nodes = list(self.nodes.values())
        busy = max(nd.busy_s for nd in nodes)
        auth, node = sum(nd.auth_s for nd in nodes), sum(nd.busy_s for nd in nodes)
        g = self.gc_clock
        return {"ordered_per_node": [nd.ordered for nd in nodes], "nacks_per_node": [nd.nacks for nd in nodes],
                "bad_propagates": sum(nd.bad_propagates for nd in nodes),
                "verifies": sum(nd.verifies for nd in nodes), "auth_calls": sum(nd.auth_calls for nd in nodes),
                "early_handovers": sum(nd.early_handovers for nd in nodes),
                "wall_s": wall_s, "ordered_req_per_s_one_process": n_reqs / wall_s,
                "max_node_busy_s": busy, "ordered_req_per_s_parallel_nodes": n_reqs / busy,
                "auth_share_of_node_time": auth / node,
                # the cyclic GC's time, in total and the part that landed inside
                # authentication windows; the share with every collection taken
                # out of both node time and authentication time
                "gc_share_of_node_time": g.total_s / node, "gc_in_auth_s": g.in_auth_s,
                "auth_share_excluding_gc": (auth - g.in_auth_s) / max(node - g.total_s, 1e-12),
                "latency_ms": latency_summary(nodes)}


def latency_summary(nodes):
    """p50 / p99 / max request latency in ms over every (request, node) pair."""
    out = {}
    for kind, what in (("monitor", "forwarded (f+1 PROPAGATEs, the Monitor's start) -> ordered"),
                       ("receipt", "prod that read the request off the node's inbox -> ordered"),
                       ("submit", "client submission -> ordered")):
        v = sorted(x for nd in nodes for x in nd.lat[kind])
        if not v:
            continue
        q = lambda f: 1e3 * v[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
        out[kind] = {"p50": q(0.50), "p99": q(0.99), "max": 1e3 * v[-1], "mean": 1e3 * sum(v) / len(v),
                     "samples": len(v), "what": what}
    return out

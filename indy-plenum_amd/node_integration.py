"""Node-side batching of request authentication.

In the reference every client REQUEST and every PROPAGATE is authenticated one
message at a time, inside the message loop of the Node's single Looper thread:

  Node.serviceClientMsgs -> clientstack.service -> handleOneClientMsg
      -> validateClientMsg -> verifySignature(cMsg)        plenum/server/node.py:1646-1743
  Node.serviceNodeMsgs -> nodestack.service -> handleOneNodeMsg
      -> validateNodeMsg -> verifySignature(Propagate)     plenum/server/node.py:1553-1620
  Node.verifySignature -> ReqAuthenticator.authenticate    plenum/server/node.py:2575-2599

so each request costs one libsodium verify per node for the client copy and one
per PROPAGATE received (n verifies per node, n^2 per pool).  ProdAuthBatch
gathers the messages of one prod (<= DEFAULT_LISTENER_QUOTA per listener read,
stp_core/config.py:28) and authenticates all of them with ONE
ReqAuthenticator.authenticate_batch call (one GPU launch); per-message
processing then continues in the original order with each message's own
verdict, so the PRE/POST_SIG_VERIFICATION hooks and every exception path see
exactly what the sequential loop would have produced.
"""
from typing import Callable, List, Optional, Sequence, Tuple

from .req_authenticator import ReqAuthenticator

DEFAULT_LISTENER_QUOTA = 100  # stp_core/config.py:28


class ProdAuthBatch:
    """Authenticate the request payloads of one prod in one batch.

    add(req_dict) -> ticket; run() once; then result(ticket) returns the set of
    identifiers ReqAuthenticator.authenticate would return, or raises the
    exception it would raise.
    """

    def __init__(self, authenticator: ReqAuthenticator):
        self._auth = authenticator
        self._reqs = []
        self._res = None

    def add(self, req) -> int:
        if self._res is not None:
            raise RuntimeError("batch already authenticated")
        self._reqs.append(req)
        return len(self._reqs) - 1

    def __len__(self):
        return len(self._reqs)

    def run(self):
        self._res = self._auth.authenticate_batch(self._reqs) if self._reqs else []
        return self

    def result(self, ticket: int):
        r = self._res[ticket]
        if isinstance(r, BaseException):
            raise r
        return r


def authenticate_prod(authenticator: ReqAuthenticator, client_msgs: Sequence[Tuple[dict, str]],
                      propagates: Sequence[Tuple[dict, str]],
                      on_client: Callable[[dict, str, object], None],
                      on_propagate: Callable[[dict, str, object], None],
                      batched: bool = True):
    """Process one prod's client REQUESTs and PROPAGATEs (each (payload, frm)).

    on_client / on_propagate receive (msg, frm, outcome) in arrival order, where
    outcome is the identifier set or the exception verifySignature would raise.
    batched=False is the reference's one-at-a-time behaviour (for comparison).
    """
    def req_of(p):
        return p["request"]

    if not batched:
        for msg, frm in propagates:
            on_propagate(msg, frm, _outcome(lambda: authenticator.authenticate(req_of(msg))))
        for msg, frm in client_msgs:
            on_client(msg, frm, _outcome(lambda: authenticator.authenticate(msg)))
        return
    b = ProdAuthBatch(authenticator)
    tp = [b.add(req_of(msg)) for msg, _frm in propagates]
    tc = [b.add(msg) for msg, _frm in client_msgs]
    b.run()
    for (msg, frm), t in zip(propagates, tp):
        on_propagate(msg, frm, _outcome(lambda: b.result(t)))
    for (msg, frm), t in zip(client_msgs, tc):
        on_client(msg, frm, _outcome(lambda: b.result(t)))


class PendingProd:
    """One prod's REQUESTs and PROPAGATEs submitted for authentication (and
    their request digests) without waiting: finish() hands each message its
    outcome in arrival order, as authenticate_prod does -- at the end of the
    same prod if ready() says the GPU is already done, else one prod later."""

    def __init__(self, authenticator: ReqAuthenticator, client_msgs, propagates, digests: bool = True):
        self.client_msgs, self.propagates = list(client_msgs), list(propagates)
        self.t_read = 0.0  # when the messages were read (the caller's clock), for latency bookkeeping
        self.reqs = [m["request"] for m, _frm in self.propagates] + [m for m, _frm in self.client_msgs]
        self._pending = authenticator.authenticate_batch_submit(self.reqs, digests=digests) if self.reqs else None

    def ready(self):
        """True when finish() will not wait for the GPU: the Node may then hand
        the prod over at once instead of at its next prod."""
        return self._pending is None or self._pending.ready()

    def digests(self, digest_fn=None):
        """Request.getDigest of every request (propagates first): the device's,
        and digest_fn's for the ones it did not hash."""
        if self._pending is None:
            return []
        d = list(self._pending.digests())
        rest = [k for k, x in enumerate(d) if x is None]
        if rest:
            if digest_fn is None:
                raise ValueError("digests missing and no digest_fn")
            for k, x in zip(rest, digest_fn([self.reqs[k] for k in rest])):
                d[k] = x
        return d

    def finish(self, on_client, on_propagate):
        res = self._pending.result() if self._pending is not None else []
        it = iter(res)
        for msg, frm in self.propagates:
            on_propagate(msg, frm, _as_outcome(next(it)))
        for msg, frm in self.client_msgs:
            on_client(msg, frm, _as_outcome(next(it)))


def _as_outcome(r):
    """authenticate_batch's per-request result: the identifier set, or the
    exception instance verifySignature would raise."""
    return r


def _outcome(f):
    try:
        return f()
    except Exception as ex:  # the exception verifySignature would raise, as a value
        return ex


def failed(outcome) -> Optional[BaseException]:
    return outcome if isinstance(outcome, BaseException) else None


__all__: List[str] = ["DEFAULT_LISTENER_QUOTA", "PendingProd", "ProdAuthBatch", "authenticate_prod", "failed"]

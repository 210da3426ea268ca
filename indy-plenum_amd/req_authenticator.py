"""ReqAuthenticator (plenum/server/req_authenticator.py:11-55) plus
authenticate_batch, the entry point a Node's client-inbox batch goes through
(SURVEY.md section 8b).

authenticate_batch(reqs) returns, for each request, exactly what
authenticate(req) returns or raises (the exception instance in place of a
raise): query short-circuit, registration order, deepcopy per authenticator,
union of identifiers, NoAuthenticatorFound.  Authenticators are applied in
order; each batch-capable one (authenticate_batch) sees all requests still
alive at its position in one call, i.e. one GPU launch per authenticator.
"""
import gc
import threading
from contextlib import contextmanager
from copy import deepcopy
from typing import Optional

from .client_authn import ClientAuthNr
from .constants import OPERATION, TXN_TYPE
from .exceptions import InsufficientCorrectSignatures, NoAuthenticatorFound


_gc_lock = threading.Lock()
_gc_depth = 0       # paused sections in progress, over all threads
_gc_was = False     # GC state when the first of them began


GC_PAUSE_MIN = 4096  # batches smaller than this leave the GC alone


@contextmanager
def gc_paused_for(n):
    """gc_paused for a batch of n requests; nothing for a small one.  A large
    batch makes tens of thousands of containers, whose allocations would
    trigger repeated collections over every live object of the node; a Node
    prod's batch (a few hundred requests) makes a few hundred, and pausing then
    only moves a collection the node's own allocations triggered to the pause's
    end, inside the batch call."""
    if n < GC_PAUSE_MIN:
        yield
        return
    with gc_paused():
        yield


@contextmanager
def gc_paused():
    """Pause the cyclic GC while a batch makes one small container per request
    (identifier sets, lists): at node scale the allocations otherwise trigger
    repeated collections over every live object; the young objects are
    collected once, after.  The GC flag is process-global and batches may run
    on several threads at once (the pool's overlap mode), so the pause is
    counted under a lock: the first section to begin records the state, the
    last one to end restores it."""
    global _gc_depth, _gc_was
    with _gc_lock:
        if _gc_depth == 0:
            _gc_was = gc.isenabled()
            gc.disable()
        _gc_depth += 1
    try:
        yield
    finally:
        with _gc_lock:
            _gc_depth -= 1
            if _gc_depth == 0 and _gc_was:
                gc.enable()


class ReqAuthenticator:
    """Ordered list of authenticators; the first one is the core authenticator."""

    def __init__(self):
        self._authenticators = []

    def register_authenticator(self, authenticator: ClientAuthNr):
        self._authenticators.append(authenticator)

    def authenticate(self, req_data):
        identifiers = set()
        typ = req_data.get(OPERATION, {}).get(TXN_TYPE)
        for authenticator in self._authenticators:
            if authenticator.is_query(typ):
                return set()
            if not (authenticator.is_write(typ) or authenticator.is_action(typ)):
                continue
            rv = authenticator.authenticate(deepcopy(req_data)) or set()
            identifiers.update(rv)
        if not identifiers:
            raise NoAuthenticatorFound
        return identifiers

    def authenticate_batch(self, reqs):
        with gc_paused():
            return self._authenticate_batch(reqs)

    def _single_stock_plan(self, reqs):
        """Fast path for the usual node set-up, one authenticator whose batch path
        is the stock read-only one: list-comprehension passes only, the type
        predicates evaluated once per distinct type.  -> (authenticator, todo,
        kinds) or None = use the general path (several authenticators, a
        malformed request, an unhashable type, a predicate that raises)."""
        if len(self._authenticators) != 1:
            return None
        a = self._authenticators[0]
        ro = getattr(a, "batch_reads_only", None)
        if not hasattr(a, "authenticate_batch") or ro is None or not ro():
            return None
        try:
            typs = [req.get(OPERATION, {}).get(TXN_TYPE) for req in reqs]
            kinds = {t: (0 if a.is_query(t) else (2 if a.is_write(t) or a.is_action(t) else 1)) for t in set(typs)}
        except Exception:
            return None
        kd = [kinds[t] for t in typs]
        return a, [k for k, x in enumerate(kd) if x == 2], kd

    @staticmethod
    def _single_stock_out(kd, todo, results):
        out = [set() if x == 0 else None for x in kd]
        for k, rv in zip(todo, results):
            # authenticate(): identifiers.update(rv or set()); none -> NoAuthenticatorFound
            out[k] = rv if isinstance(rv, BaseException) else (set(rv) if rv else NoAuthenticatorFound())
        for k, x in enumerate(kd):
            if x == 1:
                out[k] = NoAuthenticatorFound()
        return out

    def _single_stock(self, reqs):
        plan = self._single_stock_plan(reqs)
        if plan is None:
            return None
        a, todo, kd = plan
        return self._single_stock_out(kd, todo, a.authenticate_batch([reqs[k] for k in todo]))

    def authenticate_batch_submit(self, reqs, digests: bool = False):
        """Asynchronous authenticate_batch (the Node's prod keeps going while the
        GPU verifies): -> PendingAuth whose result() is authenticate_batch(reqs)
        and whose digests() holds Request.getDigest for the requests the device
        hashed (None elsewhere).  Only the single stock authenticator submits
        asynchronously; any other set-up is authenticated at once."""
        from .client_authn import PendingAuth
        native = self._native_submit(reqs, digests)
        if native is not None:
            return native
        plan = self._single_stock_plan(reqs)
        if plan is None or not hasattr(plan[0], "authenticate_batch_submit"):
            out = self.authenticate_batch(reqs)
            return PendingAuth(lambda: (out, [None] * len(reqs)))
        a, todo, kd = plan
        sub = [reqs[k] for k in todo]
        with gc_paused():
            p = a.authenticate_batch_submit(sub, digests=digests)

        def finish():
            with gc_paused():
                res = p.result()
                out = self._single_stock_out(kd, todo, res)
            dig = [None] * len(reqs)
            for k, d in zip(todo, p.digests()):
                dig[k] = d
            return out, dig
        return PendingAuth(finish, p.ready if hasattr(p, "ready") else (lambda: False))

    def _native_submit(self, reqs, digests):
        """The whole submission natively (_edvhost.req_auth_submit: the type
        routing of authenticate() and CoreAuthNr's fast path, one queued device
        call) for the usual node: one stock CoreAuthNr whose type predicates are
        the stock ones.  None = not applicable."""
        from .client_authn import CoreAuthMixin, PendingAuth, DidVerifier, _edvhost
        from . import edv
        if len(self._authenticators) != 1 or _edvhost is None:
            return None
        a = self._authenticators[0]
        cls = type(a)
        if not (isinstance(a, CoreAuthMixin) and a.batch_reads_only() and a._stock(DidVerifier)
                and edv.native_batch_enabled()
                and cls.is_query is CoreAuthMixin.is_query and cls.is_write is CoreAuthMixin.is_write
                and getattr(cls.is_action, "__func__", None) is CoreAuthMixin.is_action.__func__
                and cls.authenticate_batch_submit is CoreAuthMixin.authenticate_batch_submit):
            return None
        submit, wait = edv.async_addresses()
        with gc_paused_for(len(reqs)):
            h = _edvhost.req_auth_submit(reqs, a.clients, a.excluded_from_signing, submit, wait, edv.batch_device(),
                                         edv.PREP_THREADS, a._state_nyms(reqs), digests and a.device_digests_ok(),
                                         (a.query_types, a.write_types, cls.action_types))

        def finish():
            with gc_paused_for(len(reqs)):
                out, slow, general, digs = _edvhost.req_auth_finish(h, NoAuthenticatorFound,
                                                                   InsufficientCorrectSignatures)
                if slow:
                    res = a._batch_planned([reqs[k] for k in slow], [None] * len(slow), DidVerifier)
                    for k, rv in zip(slow, res):
                        out[k] = rv if isinstance(rv, BaseException) else (set(rv) if rv else NoAuthenticatorFound())
                if general:
                    for k, r in zip(general, self._authenticate_batch([reqs[k] for k in general])):
                        out[k] = r
            return out, (digs if digs is not None else [None] * len(reqs))
        return PendingAuth(finish, lambda: _edvhost.batch_ready(h, edv.query_address()))

    def _authenticate_batch(self, reqs):
        fast = self._single_stock(reqs)
        if fast is not None:
            return fast
        n = len(reqs)
        out = [None] * n
        typs = [None] * n
        alive = []  # requests still being processed (no result yet)
        for k, req in enumerate(reqs):
            try:
                typs[k] = req.get(OPERATION, {}).get(TXN_TYPE)
            except Exception as ex:  # malformed operation: authenticate() would raise the same
                out[k] = ex
                continue
            alive.append(k)
        idents = {}  # k -> union of the identifier sets returned so far
        for authenticator in self._authenticators:
            if not alive:
                break
            # is_query / is_write / is_action once per distinct type (pure predicates
            # of the type in the reference: client_authn.py:185-193)
            def kind(t):
                return 0 if authenticator.is_query(t) else \
                    (2 if authenticator.is_write(t) or authenticator.is_action(t) else 1)
            kinds = {}
            still, todo = [], []
            for k in alive:
                t = typs[k]
                try:
                    kd, cache = kinds.get(t), True
                except TypeError:  # an unhashable type value: evaluate it directly
                    kd, cache = None, False
                if kd is None:
                    try:
                        kd = kind(t)
                    except Exception as ex:  # what authenticate() raises for this request
                        out[k] = ex
                        continue
                    if cache:
                        kinds[t] = kd
                if kd == 0:
                    out[k] = set()
                    continue
                still.append(k)
                if kd == 2:
                    todo.append(k)
            alive = still
            if not todo:
                continue
            if hasattr(authenticator, "authenticate_batch"):
                # the reference deep-copies per authenticator (req_authenticator.py:39) so a
                # plugin cannot alter the request; the stock batch path never mutates it
                ro = getattr(authenticator, "batch_reads_only", None)
                if ro is not None and ro():
                    results = authenticator.authenticate_batch([reqs[k] for k in todo])
                else:
                    results = authenticator.authenticate_batch([deepcopy(reqs[k]) for k in todo])
            else:
                results = []
                for k in todo:
                    try:
                        results.append(authenticator.authenticate(deepcopy(reqs[k])))
                    except Exception as ex:
                        results.append(ex)
            failed = False
            for k, rv in zip(todo, results):
                if isinstance(rv, BaseException):
                    out[k] = rv
                    failed = True
                elif rv:
                    cur = idents.get(k)
                    if cur is None:
                        idents[k] = set(rv)
                    else:
                        cur.update(rv)
            if failed:
                alive = [k for k in alive if out[k] is None]
        for k in alive:
            out[k] = idents.get(k) or NoAuthenticatorFound()
        return out

    @property
    def core_authenticator(self):
        if not self._authenticators:
            raise RuntimeError('No authenticator registered yet')
        return self._authenticators[0]

    def get_authnr_by_type(self, authnr_type) -> Optional[ClientAuthNr]:
        for authnr in self._authenticators:
            if isinstance(authnr, authnr_type):
                return authnr

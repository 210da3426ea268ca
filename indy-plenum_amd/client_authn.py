"""Client authenticators (plenum/server/client_authn.py:25-258) with a batch
entry point that sends every signature of a client-inbox batch to the GPU in
ONE edv call.

Per-request semantics are the reference's, exactly:
  NaclAuthNr.authenticate_multi   client_authn.py:83-113
    - threshold defaults to len(signatures); fewer signatures -> InsufficientSignatures
    - in dict order: b58decode(sig) (any error -> InvalidSignatureFormat),
      serializeForSig, getVerkey (None -> CouldNotAuthenticate), verifier(...),
      verify; stop once `threshold` correct signatures are collected, else
      InsufficientCorrectSignatures(correct, threshold)
  CoreAuthMixin.authenticate      client_authn.py:211-246
authenticate_batch runs that loop in three phases: (1) host prep of every
signature position, recording the exception a position would raise instead of
raising it; (2) one GPU batch for all verify calls; (3) replay of the sequential
loop per request over the precomputed verdicts, so exception precedence,
early break and the returned identifier lists are unchanged.  Work done in
phase 1 for positions the sequential loop would never reach is pure (base58,
serialisation, state lookups) and its results are discarded.
"""
import json
from abc import abstractmethod
from hashlib import sha256
from typing import Dict

from . import base58
from . import edv

try:  # native host prep (csrc/edv_host.cpp, row f-1)
    from . import _edvhost
except ImportError:  # pragma: no cover - the in-tree build always provides it
    _edvhost = None
from .constants import (ACTION_TYPES, FEES, IDENTIFIER, QUERY_TYPES, ROLE, SIGNATURE, SIGNATURES, VERKEY,
                        WRITE_TYPES)
from .exceptions import (CouldNotAuthenticate, EmptyIdentifier, EmptySignature, InsufficientCorrectSignatures,
                         InsufficientSignatures, InvalidSignatureFormat, MissingIdentifier, MissingSignature,
                         UnknownIdentifier)
from .signing_serializer import serialize_msg_for_signing
from .verifier import DidVerifier, Verifier


class ClientAuthNr:
    """Interface for client authenticators (client_authn.py:25-78)."""

    @abstractmethod
    def authenticate(self, msg: Dict, identifier: str = None, signature: str = None) -> str:
        """Authenticate msg; return the identifier or raise a SigningException."""

    @abstractmethod
    def authenticate_multi(self, msg: Dict, signatures: Dict[str, str], threshold: int = None):
        """Return the identifiers whose signatures verified; raise if threshold is not met."""

    @abstractmethod
    def addIdr(self, identifier, verkey, role=None):
        """Register an identifier and its verification key."""

    @abstractmethod
    def getVerkey(self, identifier):
        """The verification key for an identifier."""


class PendingAuth:
    """A batch whose verdicts (and optional request digests) are still on the
    way: result() -> the per-request list authenticate_batch returns;
    digests() -> per request the Request.getDigest hex string or None.  The
    first call waits; both may be called any number of times."""

    __slots__ = ("_finish", "_res", "_ready")

    def __init__(self, finish, ready=None):
        self._finish = finish
        self._res = None
        self._ready = ready  # () -> bool: the device is done (None: the work was done at submission)

    def _get(self):
        if self._res is None:
            self._res = self._finish()
            self._finish = self._ready = None
        return self._res

    def ready(self):
        """True when result() will not wait for the GPU (it may still build the
        per-request results); False while the batch is on the device."""
        return self._res is not None or self._ready is None or self._ready()

    def result(self):
        return self._get()[0]

    def digests(self):
        return self._get()[1]


class _Raise:
    """A recorded exception: raised at replay time only if the sequential loop reaches it."""

    __slots__ = ("exc", "cause")

    def __init__(self, exc, cause=None):
        self.exc = exc
        self.cause = cause

    def fire(self):
        if self.cause is not None:
            raise self.exc from self.cause
        raise self.exc


class _Plan:
    """Phase-1 result for one authenticate_multi call."""

    __slots__ = ("threshold", "steps", "early")

    def __init__(self, threshold, steps, early=None):
        self.threshold = threshold
        self.steps = steps      # list of (_Raise) or (idr, vr, sig_bytes, ser, job_index)
        self.early = early      # _Raise raised before the loop (InsufficientSignatures)


class NaclAuthNr(ClientAuthNr):

    def authenticate_multi(self, msg: Dict, signatures: Dict[str, str], threshold: int = None,
                           verifier: Verifier = DidVerifier):
        return self.authenticate_multi_batch([(msg, signatures, threshold, verifier)], raise_single=True)[0]

    # ---------------------------------------------------------------- batch
    def _plan_multi(self, msg, signatures, threshold, verifier, jobs):
        num_sigs = len(signatures)
        if threshold is not None:
            if num_sigs < threshold:
                return _Plan(threshold, [], _Raise(InsufficientSignatures(num_sigs, threshold)))
        else:
            threshold = num_sigs
        steps = []
        for idr, sig in signatures.items():
            try:
                sig = base58.b58decode(sig)
            except Exception as ex:
                steps.append(_Raise(InvalidSignatureFormat(), ex))
                continue
            try:
                ser = self.serializeForSig(msg, identifier=idr)
                verkey = self.getVerkey(idr)
                if verkey is None:
                    raise CouldNotAuthenticate('Can not find verkey for {}'.format(idr))
                vr = verifier(verkey, identifier=idr)
            except Exception as ex:  # raised by the reference at this position
                steps.append(_Raise(ex))
                continue
            key = vr.batch_key() if hasattr(vr, "batch_key") else None
            if hasattr(vr, "batch_key"):
                if key is None:
                    steps.append((idr, vr, sig, ser, -1))        # no key: verify() is False
                else:
                    steps.append((idr, vr, sig, ser, len(jobs)))
                    jobs.append((sig, ser, key))
            else:
                steps.append((idr, vr, sig, ser, None))          # foreign verifier: call it
        return _Plan(threshold, steps)

    @staticmethod
    def _replay(plan, verdicts):
        if plan.early is not None:
            plan.early.fire()
        correct_sigs_from = []
        for st in plan.steps:
            if isinstance(st, _Raise):
                st.fire()
            idr, vr, sig, ser, j = st
            if j is None:
                ok = vr.verify(sig, ser)
            elif j < 0:
                ok = False
            else:
                ok = verdicts[j]
            if ok:
                correct_sigs_from.append(idr)
                if len(correct_sigs_from) == plan.threshold:
                    break
        else:
            raise InsufficientCorrectSignatures(len(correct_sigs_from), plan.threshold)
        return correct_sigs_from

    def authenticate_multi_batch(self, calls, raise_single=False):
        """calls: list of (msg, signatures, threshold, verifier).  Returns one
        entry per call: the identifier list, or the exception instance the
        reference's authenticate_multi would have raised (re-raised directly
        when raise_single is set and there is one call)."""
        jobs = []
        plans = [self._plan_multi(msg, signatures, threshold, verifier or DidVerifier, jobs)
                 for msg, signatures, threshold, verifier in calls]
        return self._run_plans(plans, jobs, raise_single)

    def _run_plans(self, plans, jobs, raise_single=False):
        """Phase 2 (one device call for every job) and phase 3 (replay)."""
        verdicts = edv.open_batch(jobs) if jobs else []
        out = []
        for plan in plans:
            if raise_single:
                out.append(self._replay(plan, verdicts))
                continue
            try:
                out.append(self._replay(plan, verdicts))
            except Exception as ex:
                out.append(ex)
        return out

    @abstractmethod
    def addIdr(self, identifier, verkey, role=None):
        pass

    @abstractmethod
    def getVerkey(self, identifier):
        pass

    def serializeForSig(self, msg, identifier=None, topLevelKeysToIgnore=None):
        return serialize_msg_for_signing(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)


def nym_to_state_key(nym: str) -> bytes:
    """DomainRequestHandler.nym_to_state_key (plenum/server/domain_req_handler.py:166-167)."""
    return sha256(nym.encode()).digest()


def get_nym_details(state, nym, isCommitted: bool = True):
    """DomainRequestHandler.getNymDetails (domain_req_handler.py:158-163): JSON
    value under sha256(nym) in the state, {} if absent."""
    data = state.get(nym_to_state_key(nym), isCommitted) if state is not None else None
    if not data:
        return {}
    return json.loads(data.decode() if isinstance(data, (bytes, bytearray)) else data)


class SimpleAuthNr(NaclAuthNr):
    """In-memory identifiers, then the (uncommitted) state (client_authn.py:128-168)."""

    def __init__(self, state=None):
        self.clients = {}  # type: Dict[str, Dict]
        self.state = state

    def addIdr(self, identifier, verkey, role=None):
        self.clients[identifier] = {VERKEY: verkey, ROLE: role}

    def getVerkey(self, identifier):
        nym = self.clients.get(identifier)
        if not nym:
            nym = get_nym_details(self.state, identifier, isCommitted=False)
            if not nym:
                raise UnknownIdentifier(identifier)
        return nym.get(VERKEY)

    def authenticate(self, msg: Dict, identifier: str = None, signature: str = None):
        signatures = {identifier: signature}
        return self.authenticate_multi(msg, signatures=signatures)


class CoreAuthMixin:
    excluded_from_signing = {SIGNATURE, SIGNATURES, FEES}
    write_types = WRITE_TYPES
    query_types = QUERY_TYPES
    action_types = ACTION_TYPES

    def is_query(self, typ):
        return typ in self.query_types

    def is_write(self, typ):
        return typ in self.write_types

    @classmethod
    def is_action(cls, typ):
        return typ in cls.action_types

    @staticmethod
    def _extract_signature(msg):
        if SIGNATURE not in msg:
            raise MissingSignature
        if not msg[SIGNATURE]:
            raise EmptySignature
        return msg[SIGNATURE]

    @staticmethod
    def _extract_identifier(msg):
        if IDENTIFIER not in msg:
            raise MissingIdentifier
        if not msg[IDENTIFIER]:
            raise EmptyIdentifier
        return msg[IDENTIFIER]

    def _prepare(self, req_data, identifier=None, signature=None):
        """The pre-loop part of authenticate (client_authn.py:222-244):
        -> (to_serialize, signatures) or raises."""
        to_serialize = {k: v for k, v in req_data.items() if k not in self.excluded_from_signing}
        if req_data.get(SIGNATURE) is None and req_data.get(SIGNATURES) is None and signature is None:
            raise MissingSignature
        if req_data.get(IDENTIFIER) and (req_data.get(SIGNATURE) or signature):
            try:
                identifier = identifier or self._extract_identifier(req_data)
                signature = signature or self._extract_signature(req_data)
                signatures = {identifier: signature}
            except Exception as ex:
                if ex in (MissingSignature, EmptySignature, MissingIdentifier, EmptyIdentifier):
                    ex = ex(req_data.get(IDENTIFIER), req_data.get(SIGNATURE))
                raise ex
        else:
            signatures = req_data[SIGNATURES]
        return to_serialize, signatures

    def authenticate(self, req_data, identifier: str = None, signature: str = None,
                     verifier: Verifier = DidVerifier):
        to_serialize, signatures = self._prepare(req_data, identifier, signature)
        return self.authenticate_multi(to_serialize, signatures=signatures, verifier=verifier)

    def authenticate_batch(self, reqs, verifier: Verifier = DidVerifier):
        """Batch form of authenticate over a list of request dicts: one GPU
        call for all of them.  Returns, per request, the identifier list or
        the exception instance authenticate() would raise.

        Requests on the common path (one signature, identifier present, verkey
        in the in-memory `clients` map, DidVerifier giving a 32-byte key) are
        prepared natively in one call (_edvhost.prep_core_batch, row f-1); every
        other request goes through the Python plan, which raises exactly what
        the reference raises."""
        n = len(reqs)
        whole = self._native_batch(reqs, verifier)
        if whole is not None:
            # one native call did host prep + the GPU verify for the common path
            out, slow, rejected = whole
            for k in rejected:
                out[k] = InsufficientCorrectSignatures(0, 1)
            if slow:
                sub = [reqs[k] for k in slow]
                for k, r in zip(slow, self._batch_planned(sub, [None] * len(sub), verifier)):
                    out[k] = r
            return out
        return self._batch_planned(reqs, self._native_prep(reqs, verifier), verifier)

    def _batch_planned(self, reqs, fast, verifier):
        """authenticate_batch over per-request native prep results (`fast`,
        None entries take the Python plan): one open_batch call, then replay."""
        n = len(reqs)
        out = [None] * n
        if fast is None:
            fast = [None] * n
        # fast requests: jobs 0..F-1, result [idr] or InsufficientCorrectSignatures(0, 1)
        # (threshold None -> 1 signature), exactly what the replay of their plan gives
        fast_idx = [k for k in range(n) if fast[k] is not None]
        jobs = [fast[k][1:] for k in fast_idx]
        plans, where = [], []
        for k in range(n):
            if fast[k] is not None:
                continue
            try:
                to_serialize, signatures = self._prepare(reqs[k])
            except Exception as ex:
                out[k] = ex
                continue
            plans.append(self._plan_multi(to_serialize, signatures, None, verifier or DidVerifier, jobs))
            where.append(k)
        verdicts = edv.open_batch(jobs) if jobs else []
        for j, k in enumerate(fast_idx):
            out[k] = [fast[k][0]] if verdicts[j] else InsufficientCorrectSignatures(0, 1)
        for k, plan in zip(where, plans):
            try:
                out[k] = self._replay(plan, verdicts)
            except Exception as ex:
                out[k] = ex
        return out

    def _stock(self, verifier):
        """True when this authenticator and verifier are the stock ones (an
        override of any step the native code restates keeps the Python path)."""
        cls = type(self)
        return not (_edvhost is None or verifier is not DidVerifier
                    or not isinstance(getattr(self, "clients", None), dict)
                    or cls._prepare is not CoreAuthMixin._prepare
                    or cls.serializeForSig is not CoreAuthMixin.serializeForSig
                    or cls._plan_multi is not NaclAuthNr._plan_multi
                    or cls.getVerkey is not SimpleAuthNr.getVerkey
                    or base58._native is None)

    def device_digests_ok(self):
        """Device request digests (digest_is_signing_bytes in csrc/edv_host.cpp)
        treat exactly signature / signatures / fees as the keys outside the
        signing bytes, i.e. the stock excluded_from_signing (client_authn.py:174);
        with any other set the signing bytes are not signingState's bytes."""
        return set(self.excluded_from_signing) == CoreAuthMixin.excluded_from_signing

    def _native_prep(self, reqs, verifier):
        """_edvhost.prep_core_batch for the stock authenticator, else None."""
        if not self._stock(verifier):
            return None
        return _edvhost.prep_core_batch(reqs, self.clients, self.excluded_from_signing)

    def _native_batch(self, reqs, verifier):
        """_edvhost.auth_core_batch (host prep on PREP_THREADS threads + one
        edv_verify_batch call, GIL released) -> (out, slow, rejected), for the
        stock authenticator and the stock verify entry point, else None."""
        if not self._stock(verifier) or not edv.native_batch_enabled():
            return None
        return _edvhost.auth_core_batch(reqs, self.clients, self.excluded_from_signing, edv.verify_address(),
                                        edv.BATCH_DEVICE_MASK, edv.PREP_THREADS, self._state_nyms(reqs))

    def authenticate_batch_submit(self, reqs, verifier: Verifier = DidVerifier, digests: bool = False):
        """Asynchronous authenticate_batch: host prep now and the device call
        queued (edv_verify_digest_batch_async), so the caller keeps working while
        the GPU verifies; PendingAuth.result() waits and returns what
        authenticate_batch returns.  digests=True also asks the device for
        Request.getDigest (request.py:71-72) of every request whose signing bytes
        are its signingState serialization (PendingAuth.digests(); None entries
        for the rest).  Without the stock native path the work is done here, at
        once, and the PendingAuth only hands it over."""
        if self._stock(verifier) and edv.native_batch_enabled():
            submit, wait = edv.async_addresses()
            h = _edvhost.auth_core_submit(reqs, self.clients, self.excluded_from_signing, submit, wait,
                                          edv.batch_device(), edv.PREP_THREADS, self._state_nyms(reqs),
                                          digests and self.device_digests_ok())
            return PendingAuth(lambda: self._finish_native(reqs, h, verifier),
                               lambda: _edvhost.batch_ready(h, edv.query_address()))
        out = self.authenticate_batch(reqs, verifier)
        return PendingAuth(lambda: (out, [None] * len(reqs)))

    def _finish_native(self, reqs, handle, verifier):
        out, slow, rejected, digs = _edvhost.auth_core_finish(handle)
        for k in rejected:
            out[k] = InsufficientCorrectSignatures(0, 1)
        if slow:
            sub = [reqs[k] for k in slow]
            for k, r in zip(slow, self._batch_planned(sub, [None] * len(sub), verifier)):
                out[k] = r
        return out, (digs if digs is not None else [None] * len(reqs))

    # below this many state keys hashlib beats a device round trip
    STATE_KEYS_ON_DEVICE = 512

    def _state_nyms(self, reqs):
        """The NYMs getVerkey would read from the uncommitted state for this
        batch (client_authn.py:148-160 -> domain_req_handler.py:158-167): every
        string identifier whose `clients` entry is missing or falsy.  Their state
        keys (nym_to_state_key) come from one SHA-256 batch (row f-3), then one
        state.get(key, isCommitted=False) each, as the reference does per
        request.  -> {identifier: nym dict} holding non-empty dicts only (any
        other value -- absent, empty, not a JSON object -- stays with the Python
        plan, which raises what the reference raises), or None without a state."""
        state = self.state
        if state is None:
            return None
        if _edvhost is not None and hasattr(state, "get"):
            # the same reads natively (state keys by a CPU SHA-256, the usual flat
            # JSON value parsed in C, anything else through json.loads)
            return _edvhost.state_nyms(reqs, self.clients, state.get, json.loads) or None
        return self._state_nyms_py(reqs)

    def _state_nyms_py(self, reqs):
        """Python restatement of _edvhost.state_nyms (tests pin one against the other)."""
        state = self.state
        clients = self.clients
        idrs = []
        seen = set()
        for r in reqs:
            if type(r) is dict:
                i = r.get(IDENTIFIER)
                if type(i) is str and i and i not in seen and not clients.get(i):
                    seen.add(i)
                    try:
                        i.encode()
                    except UnicodeEncodeError:
                        # e.g. a lone surrogate: that request alone takes the plan,
                        # whose getVerkey raises the reference's error for it
                        continue
                    idrs.append(i)
        if not idrs:
            return None
        if len(idrs) >= self.STATE_KEYS_ON_DEVICE:
            from .digest import nym_state_keys
            keys = nym_state_keys(idrs)
        else:
            keys = [nym_to_state_key(i) for i in idrs]
        out = {}
        loads = json.loads
        for i, key in zip(idrs, keys):
            try:
                data = state.get(key, False)
                if not data:
                    continue
            except MemoryError:
                raise
            except Exception:
                continue  # a read that raises: the plan repeats it for that request alone
            try:
                nym = loads(bytes(data).decode() if isinstance(data, (bytes, bytearray)) else data)
            except Exception:
                continue
            if type(nym) is dict and nym:
                out[i] = nym
        return out

    # requests are only read, never mutated, by the stock batch path above
    def batch_reads_only(self):
        cls = type(self)
        return (cls.authenticate_batch is CoreAuthMixin.authenticate_batch
                and cls.serializeForSig is CoreAuthMixin.serializeForSig
                and cls._prepare is CoreAuthMixin._prepare)

    def serializeForSig(self, msg, identifier=None, topLevelKeysToIgnore=None):
        if not msg.get(IDENTIFIER):
            msg = {**msg, IDENTIFIER: identifier}
        return serialize_msg_for_signing(msg, topLevelKeysToIgnore=topLevelKeysToIgnore)


class CoreAuthNr(CoreAuthMixin, SimpleAuthNr):
    def __init__(self, state=None):
        SimpleAuthNr.__init__(self, state)
        CoreAuthMixin.__init__(self)


# The name the integration docs use for the batch-capable core authenticator.
GpuAuthNr = CoreAuthNr

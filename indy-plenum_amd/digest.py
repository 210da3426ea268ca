"""Request digests and NYM state keys in batches.

Same results as the reference's per-request hashing, computed by one
edv_sha256_batch call (gfx950 kernel edv_sha256_kernel) for the whole batch:

  plenum/common/request.py:71-72        Request.getDigest()
      sha256(serialize_msg_for_signing(self.signingState())).hexdigest()
  plenum/common/request.py:77-87        Request.signingState(identifier=None)
      {identifier, reqId, operation [, protocolVersion]}
  plenum/server/domain_req_handler.py:166-167   nym_to_state_key(nym)
      sha256(nym.encode()).digest()
"""
from . import _edvhost, edv
from .constants import IDENTIFIER, OPERATION, PROTOCOL_VERSION, REQ_ID, SIGNATURES
from .signing_serializer import serialize_msg_for_signing


def _identifier(req):
    """Request.identifier (request.py:110-112): the identifier, else one derived
    from the signatures (gen_idr_from_sigs, request.py:124-126: sorted DIDs joined
    by ','; like the reference, no signatures either -> AttributeError)."""
    return req.get(IDENTIFIER) or ",".join(sorted(req.get(SIGNATURES).keys()))


def signing_state(req, identifier=None):
    """Request.signingState for a request given as its dict (request.py:77-87)."""
    dct = {IDENTIFIER: identifier or _identifier(req), REQ_ID: req.get(REQ_ID), OPERATION: req.get(OPERATION)}
    if req.get(PROTOCOL_VERSION) is not None:
        dct[PROTOCOL_VERSION] = req[PROTOCOL_VERSION]
    return dct


def request_digests(reqs, device_mask: int = 0):
    """[Request.getDigest() for each request dict], one GPU batch.  The usual
    request (a dict with an identifier) is serialized natively and hashed in the
    same native call (_edvhost.request_digests, GIL released during the GPU
    call); the rest takes the Python serializer and a second batch."""
    reqs = list(reqs)
    out = _edvhost.request_digests(reqs, edv.sha256_address(), device_mask) if reqs else []
    rest = [k for k, d in enumerate(out) if d is None]
    if rest:
        for k, d in zip(rest, edv.sha256_batch([serialize_msg_for_signing(signing_state(reqs[k])) for k in rest],
                                               device_mask)):
            out[k] = d.hex()
    return out


def nym_state_keys(nyms, device_mask: int = 0):
    """[DomainRequestHandler.nym_to_state_key(nym) for each DID string], one GPU batch."""
    return edv.sha256_batch([n.encode() for n in nyms], device_mask)

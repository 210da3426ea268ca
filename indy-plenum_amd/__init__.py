"""indy-plenum_amd: MI355X (gfx950) batch Ed25519 verification for Plenum's
client-request authentication hot path.

Drop-in for the reference's authenticator plugin surface:
  ClientAuthNr / NaclAuthNr / CoreAuthNr   plenum/server/client_authn.py
  Verifier / DidVerifier                   plenum/common/verifier.py
  Verifier / VerifyKey                     stp_core/crypto/nacl_wrappers.py
  ReqAuthenticator                         plenum/server/req_authenticator.py
plus batch entry points (authenticate_batch, verify_batch) that hand a whole
client-inbox batch to the HIP kernels through the C-ABI in include/edv.h.
"""
__version__ = "0.1.0"

"""Field names and transaction types the authentication path reads
(plenum/common/types.py:23-75, plenum/common/constants.py:66-127,
plenum/common/transactions.py:14-16)."""
IDENTIFIER = 'identifier'
SIGNATURE = 'signature'
SIGNATURES = 'signatures'
FEES = 'fees'
OPERATION = 'operation'
TXN_TYPE = 'type'
VERKEY = 'verkey'
ROLE = 'role'
REQ_ID = 'reqId'
PROTOCOL_VERSION = 'protocolVersion'

NODE = "0"
NYM = "1"
GET_TXN = "3"

# CoreAuthMixin type sets (plenum/server/client_authn.py:175-183):
# PoolRequestHandler.write_types = {NODE}, DomainRequestHandler.write_types = {NYM},
# both handlers' query_types are empty, ActionReqHandler.operation_types is empty.
WRITE_TYPES = frozenset({NODE, NYM})
QUERY_TYPES = frozenset({GET_TXN})
ACTION_TYPES = frozenset()

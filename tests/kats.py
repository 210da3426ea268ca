"""Signed-request known-answer fixtures held in the reference's own tests
(SURVEY.md section 4): verdicts confirmed with libsodium 1.0.18 + the reference
SigningSerializer during the survey, re-checked by tests/test_authn_host.py
against the oracle."""

# KAT-1: plenum/test/node_request/message_request/test_valid_message_request.py:74-79
KAT1_IDR = '5rArie7XKukPCaEwq5XGQJnM9Fc5aZE3M9HAPVfMU2xC'   # 32-byte cryptonym = its own verkey
KAT1_SIG = 'ZbZG68WiaK67eU3CsgpVi85jpgCztW9Yqe7D5ezDUfWbKdiPPVbWq4Tb5m4Ur3jcR5wJ8zmBUZXZudjvMN63Aa9'


def kat1_request(protocol_version=None):
    req = {'identifier': KAT1_IDR, 'signature': KAT1_SIG, 'operation': {'amount': 62, 'type': 'buy'},
           'reqId': 1499782864169193}
    if protocol_version is not None:
        req['protocolVersion'] = protocol_version
    return req


# KAT-2: plenum/test/transactions/test_new_txn_format.py:11-25 (NYM); signer verkey is the
# cryptonym of plenum/test/common/test_signers.py:37-39
KAT2_IDR = 'L5AD5g65TDQr1PPHHRoiGf'
KAT2_ABBR_VERKEY = '~Bf9Z1tKWpcJAvKJVhZhvVZ'
KAT2_CRYPTONYM = 'BPtrqHo3WyjmTNpVchEhWxp3qfDdssdFUNoM8kmKoEWw'
KAT2_SIG = '3SyRto3MGcBy1o4UmHoDezy1TJiNHDdU9o7TjHtYcSqgtpWzejMoHDrz3dpT93Xe8QXMF2tJVCQTtGmebmS2DkLS'


def kat2_request(protocol_version=1):
    req = {'identifier': KAT2_IDR, 'reqId': 1513945121191691, 'signature': KAT2_SIG,
           'operation': {'dest': 'GEzcdDLhCpGCYRHW82kjHd', 'verkey': '~HmUWn928bnFT6Ephf65YXv', 'role': '101',
                         'type': '1'}}
    if protocol_version is not None:
        req['protocolVersion'] = protocol_version
    return req


# DID fixtures: plenum/test/common/test_verifier.py:6-9
SAMPLE_ABBR_VERKEY = '~8zH9ZSyZTFPGJ4ZPL5Rvxx'
SAMPLE_IDENTIFIER = '99BgFBg35BehzfSADV5nM4'
EXPECTED_VERKEY = '5SMfqc4NGeQM21NMx3cB9sqop6KCFFC1TqoGKGptdock'
ODD_LENGTH_VERKEY = 'FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF'

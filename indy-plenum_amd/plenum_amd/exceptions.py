"""The authentication exceptions of the reference (plenum/common/exceptions.py:
4-9, 28-117).

Inside a Plenum node (the reference package importable) these names ARE the
reference's classes, re-exported: what the drop-in raises is caught by the
node's own handlers -- `except BaseExc` in validateNodeMsg turning a forged
PROPAGATE into SuspiciousNode (node.py:1313-1316) and the REQNACK mapping of
validateClientMsg (node.py:1383-1397, reasonForClientFromException
node.py:2568-2571).  Without the reference package (standalone use, this
repo's tests) the same names, codes, reasons and constructor behaviour are
defined here.  InsufficientSignatures / InsufficientCorrectSignatures belong
to the authenticate_multi extension, which the reference snapshot does not
have (parity unpinned); they derive from SigningException either
way."""

import re

_NODE_NAME = re.compile(r'(\b\w+)(:(\d+))?')  # exceptions.py:125 ("Alpha-1:9701" -> "Alpha")

_NAMES = ("ReqInfo", "BaseExc", "SigningException", "CouldNotAuthenticate", "MissingSignature", "EmptySignature",
          "InvalidSignatureFormat", "InvalidSignature", "MissingIdentifier", "EmptyIdentifier",
          "UnknownIdentifier", "InvalidIdentifier", "InvalidKey", "SuspiciousNode")

try:
    import plenum.common.exceptions as _ref
    globals().update({name: getattr(_ref, name) for name in _NAMES})
    REFERENCE = True
except Exception:
    REFERENCE = False

if not REFERENCE:
    class ReqInfo:
        def __init__(self, identifier=None, reqId=None):
            self.identifier = identifier
            self.reqId = reqId

    class BaseExc(Exception):
        def __str__(self):
            return "{}{}".format(self.__class__.__name__, self.args)

    class SigningException(BaseExc):
        pass

    def _signing(name, code, reason, req_info):
        """A SigningException subclass; with req_info its constructor takes
        (identifier=None, reqId=None) like ReqInfo and records no args."""
        bases = (SigningException, ReqInfo) if req_info else (SigningException,)
        ns = {"code": code, "reason": reason, "__module__": __name__}
        if req_info:
            ns["__init__"] = lambda self, *a, **k: ReqInfo.__init__(self, *a, **k)
        return type(name, bases, ns)

    CouldNotAuthenticate = _signing("CouldNotAuthenticate", 110, 'could not authenticate', True)
    MissingSignature = _signing("MissingSignature", 120, 'missing signature', False)
    EmptySignature = _signing("EmptySignature", 121, 'empty signature', True)
    InvalidSignatureFormat = _signing("InvalidSignatureFormat", 123, 'invalid signature format', True)
    InvalidSignature = _signing("InvalidSignature", 125, 'invalid signature', True)
    MissingIdentifier = _signing("MissingIdentifier", 130, 'missing identifier', False)
    EmptyIdentifier = _signing("EmptyIdentifier", 131, 'empty identifier', False)
    UnknownIdentifier = _signing("UnknownIdentifier", 133, 'unknown identifier', True)
    InvalidIdentifier = _signing("InvalidIdentifier", 135, 'invalid identifier', True)

    class InvalidKey(Exception):
        code = 142
        reason = 'invalid key'

    class SuspiciousNode(BaseExc):
        """node.py:1315 wraps an authentication failure of a node message:
        SuspiciousNode(frm, ex, msg) (exceptions.py:120-131; `suspicion` is the
        caught exception there, so code/reason come from it when present)."""

        def __init__(self, node, suspicion, offendingMsg):
            node = node.decode() if isinstance(node, bytes) else node
            self.code = suspicion.code if suspicion else None
            self.reason = suspicion.reason if suspicion else None
            m = _NODE_NAME.match(node)
            self.node = m.groups()[0] if m else node
            self.offendingMsg = offendingMsg

        def __repr__(self):
            return "Error code: {}. {}".format(self.code, self.reason)


# --- authenticate_multi extension (not in the reference snapshot) ----------
class InsufficientSignatures(SigningException):
    code = 150
    reason = 'insufficient number of signatures'

    def __init__(self, provided, required):
        super().__init__(provided, required)


class InsufficientCorrectSignatures(SigningException):
    code = 151
    reason = 'insufficient number of correct signatures'

    def __init__(self, provided, required):
        super().__init__(provided, required)


def friendlyEx(ex):
    """plenum/common/util.py:354-365: exception text with its __cause__ chain."""
    parts = []
    while ex:
        parts.append("{}".format(ex))
        ex = ex.__cause__
    return " [caused by ".join(parts) + "]" * (len(parts) - 1)


def reasonForClientFromException(ex):
    """node.py:2568-2571: the REQNACK reason a client gets."""
    return "client request invalid: {}".format(friendlyEx(ex))

"""The authentication exceptions of the reference, same names, codes, reasons
and constructor behaviour (plenum/common/exceptions.py:4-9, 28-112, 115-117),
so callers that map them (node.py:1383-1397 REQNACK via
reasonForClientFromException node.py:2568-2571; node.py:1315 SuspiciousNode)
see identical objects.  InsufficientSignatures / InsufficientCorrectSignatures
belong to the authenticate_multi extension, which the reference snapshot does
not have (parity unpinned)."""


class ReqInfo:
    def __init__(self, identifier=None, reqId=None):
        self.identifier = identifier
        self.reqId = reqId


class BaseExc(Exception):
    def __str__(self):
        return "{}{}".format(self.__class__.__name__, self.args)


class SigningException(BaseExc):
    pass


class CouldNotAuthenticate(SigningException, ReqInfo):
    code = 110
    reason = 'could not authenticate'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class MissingSignature(SigningException):
    code = 120
    reason = 'missing signature'


class EmptySignature(SigningException, ReqInfo):
    code = 121
    reason = 'empty signature'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidSignatureFormat(SigningException, ReqInfo):
    code = 123
    reason = 'invalid signature format'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidSignature(SigningException, ReqInfo):
    code = 125
    reason = 'invalid signature'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class MissingIdentifier(SigningException):
    code = 130
    reason = 'missing identifier'


class EmptyIdentifier(SigningException):
    code = 131
    reason = 'empty identifier'


class UnknownIdentifier(SigningException, ReqInfo):
    code = 133
    reason = 'unknown identifier'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidIdentifier(SigningException, ReqInfo):
    code = 135
    reason = 'invalid identifier'

    def __init__(self, *args, **kwargs):
        ReqInfo.__init__(self, *args, **kwargs)


class InvalidKey(Exception):
    code = 142
    reason = 'invalid key'


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
    cur, friendly, end = ex, "", ""
    while cur:
        if len(friendly):
            friendly += " [caused by "
            end += "]"
        friendly += "{}".format(cur)
        cur = cur.__cause__
    return friendly + end


def reasonForClientFromException(ex):
    """node.py:2568-2571: the REQNACK reason a client gets."""
    return "client request invalid: {}".format(friendlyEx(ex))

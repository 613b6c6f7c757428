"""JSON encoding of Erlang terms for the golden fixtures (data only)."""

from oracle.terms import Atom as OAtom


def enc(t):
    if isinstance(t, bool):
        return {"atom": "true" if t else "false"}
    if isinstance(t, str):                      # oracle Atom or lasp_amd Atom
        return {"atom": str.__str__(t)}
    if isinstance(t, int):
        return {"int": t}
    if isinstance(t, (bytes, bytearray)):
        return {"bin": bytes(t).hex()}
    if isinstance(t, tuple):
        return {"tuple": [enc(x) for x in t]}
    if isinstance(t, list):
        return {"list": [enc(x) for x in t]}
    raise TypeError(t)


def dec(j, atom=OAtom):
    (k, v), = j.items()
    if k == "atom":
        return True if v == "true" else False if v == "false" else atom(v)
    if k == "int":
        return v
    if k == "bin":
        return bytes.fromhex(v)
    if k == "tuple":
        return tuple(dec(x, atom) for x in v)
    if k == "list":
        return [dec(x, atom) for x in v]
    raise ValueError(k)

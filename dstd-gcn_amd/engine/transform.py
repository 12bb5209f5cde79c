"""Shape transforms used by the engine (reference engine/utils/transform.py:35-49).
Views only: no data is moved."""


def tsc_transform(data, c=3):
    """(batch, time, space * c) -> (batch, time, space, c)   (transform.py:35-41)"""
    B, T, SC = data.shape
    assert SC % c == 0
    return data.view(B, T, SC // c, c)


def tsc_inverse(data, c=3):
    """(batch, time, space, c) -> (batch, time, space * c)   (transform.py:44-49)"""
    B, T, S, C = data.shape
    assert C == c
    return data.view(B, T, S * C)


TRANSFORMS = {"tsc": (tsc_transform, tsc_inverse), "no": (None, None)}

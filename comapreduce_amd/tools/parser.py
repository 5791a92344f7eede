"""``.ini`` parameter files for run_destriper (reference Tools/ParserClass.py:4-101)
and ``Coordinates.sex2deg`` (Tools/Coordinates.py:19-32).

Parsing rules kept from the reference: '#' starts a comment; ``[Header]``
opens a section; the first of ':' or '=' splits key from value; spaces are
removed from keys and values; a value with commas becomes a list (empty items
dropped); 'None'/'True'/'False' map to None/True/False, anything float()
accepts becomes a float, the rest stays a string.  Unknown keys raise
AttributeError like the reference's ``__getitem__``.
"""
from __future__ import annotations

import re


def _convert(v):
    if v == 'None':
        return None
    if v.strip() == 'True':
        return True
    if v.strip() == 'False':
        return False
    try:
        return float(v)
    except ValueError:
        return v


class Parser:
    def __init__(self, filename):
        self.infodict = {}
        with open(filename, 'r') as f:
            self._read(f)

    def __str__(self):
        return '{' + ''.join(k + ',\n' for k in self.infodict) + '}'

    def __setitem__(self, k, v):
        self.infodict[k] = v

    def __getitem__(self, k):
        try:
            return self.infodict[k]
        except KeyError:
            raise AttributeError('Unknown key: {}'.format(k))

    def __contains__(self, k):
        return k in self.infodict

    def items(self):
        return self.infodict.items()

    def _read(self, lines):
        header = None
        for line in lines:
            s = line.split('#')[0].strip()
            if not s:
                continue
            if s[0] == '[' and s[-1] == ']':
                header = re.split('\\[|\\]', s)[1]
                self.infodict.setdefault(header, {})
                continue
            if ':' not in s and '=' not in s:
                raise ValueError(f'no ":" or "=" in parameter line {line!r}')
            i = s.index(':') if ':' in s else s.index('=')
            key, value = s[:i].replace(' ', ''), s[i + 1:].strip().replace(' ', '').split(',')
            if len(value) > 1:
                self.infodict[header][key] = [_convert(v) for v in value if v != '']
            else:
                self.infodict[header][key] = _convert(value[0])


def sex2deg(dms, hours=False):
    """'dd:mm:ss' -> degrees (x15 for hours); the sign is taken from the degree field."""
    d, m, s = dms.split(':')
    sign = -1 if '-' in d else 1
    out = sign * (abs(float(d)) + float(m) / 60. + float(s) / 60. ** 2)
    return out * 15. if hours else out

import builtins as _b

range, filter, map, zip = _b.range, _b.filter, _b.map, _b.zip
chr, input, open, next, round, super = _b.chr, _b.input, _b.open, _b.next, _b.round, _b.super
str, bytes, int, object, dict, list = _b.str, _b.bytes, _b.int, _b.object, _b.dict, _b.list

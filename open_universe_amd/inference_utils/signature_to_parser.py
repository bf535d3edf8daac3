"""``add_enhance_arguments`` (mirrors inference_utils/signature_to_parser.py:26-66):
argparse options generated from ``typing.get_type_hints(model.enhance)``.

This function follows the reference's own implementation closely because the
CLI contract is the function itself (the argument names, types and defaults
the reference CLI derives from the type hints).  That implementation is
Copyright 2024 LY Corporation, licensed under the Apache License, Version 2.0
(http://www.apache.org/licenses/LICENSE-2.0).
"""
import typing


def add_enhance_arguments(model, parser):
    if not (hasattr(model, "enhance") and callable(model.enhance)):
        raise ValueError("Model does not have an `enhance` method.")
    enhance_args = typing.get_type_hints(model.enhance)
    enhance_args.pop("return", None)
    default_kwargs = getattr(model, "diff_kwargs", {})
    type_casters = {}
    for key, val in enhance_args.items():
        types = typing.get_args(val)
        type_casters[key] = val if len(types) == 0 else types[0]
    group = parser.add_argument_group("enhance", "Arguments of enhance function")
    for key, type_cast in type_casters.items():
        group.add_argument(f"--{key}", default=default_kwargs.get(key, None), type=type_cast)
    return parser

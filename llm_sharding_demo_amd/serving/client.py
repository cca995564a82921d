"""Client helpers.

`generate_text` keeps the notebook helper's signature and return contract
(`/root/reference/notebook.ipynb:111-120`): the parsed JSON dict on HTTP 200,
otherwise the string "Error: {code} - {text}"; network failures return
"Request failed: {exc}".
"""
from __future__ import annotations

import os
from typing import Union

COORDINATOR_URL = os.environ.get("COORDINATOR_URL", "http://127.0.0.1:5000/generate")


def generate_text(prompt: str, max_new_tokens: int = 20, url: str = None,
                  timeout: float = 300.0, **sampling) -> Union[dict, str]:
    import requests

    payload = {"prompt": prompt, "max_new_tokens": max_new_tokens}
    payload.update({k: v for k, v in sampling.items() if v is not None})
    try:
        r = requests.post(url or COORDINATOR_URL, json=payload, timeout=timeout)
        if r.status_code == 200:
            return r.json()
        return f"Error: {r.status_code} - {r.text}"
    except requests.exceptions.RequestException as e:
        return f"Request failed: {e}"

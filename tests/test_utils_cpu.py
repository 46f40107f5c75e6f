"""CPU: make_env_and_datasets' name grammar against the reference's own
utils.py (tests/golden/names_golden.json), and the C-ABI exports of the loader."""

import json
import os

import pytest

from ogbench_amd.utils import parse_dataset_name

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'names_golden.json')


@pytest.mark.parametrize('case', json.load(open(GOLD)), ids=lambda c: c['dataset_name'])
def test_name_grammar_matches_reference(case):
    env_name, file_name, mode = parse_dataset_name(case['dataset_name'])
    assert env_name == case['env_name']
    assert file_name == case['file_name']
    assert (mode == 'oraclerep') == (case['env_kwargs'] == {'use_oracle_rep': True})

#!/bin/bash
exec bash "$(dirname "$0")/r03p.sh" 2

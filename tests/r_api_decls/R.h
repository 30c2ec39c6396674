#pragma once
/* see Rinternals.h */
